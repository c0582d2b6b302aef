"""CPU: the Zipf corpus generator (tools/iigen.c) is deterministic and keeps
the layout contract the device path relies on."""
import hashlib

import numpy as np

import ii_ctypes


def test_deterministic_and_thread_invariant():
    a, oa = ii_ctypes.zipf_corpus(3_000_000, 37, 5000, 5, threads=1)
    b, ob = ii_ctypes.zipf_corpus(3_000_000, 37, 5000, 5, threads=7)
    assert (oa == ob).all()
    assert hashlib.sha256(a.tobytes()).digest() == hashlib.sha256(b.tobytes()).digest()
    c, _ = ii_ctypes.zipf_corpus(3_000_000, 37, 5000, 6, threads=4)
    assert hashlib.sha256(a.tobytes()).digest() != hashlib.sha256(c.tobytes()).digest()


def test_layout():
    t, off = ii_ctypes.zipf_corpus(1_000_000, 100, 1000, 9, threads=4)
    assert off[0] == 0 and off[-1] == 1_000_000
    assert (np.diff(off.astype(np.int64)) >= 0).all()
    ws = set(b" \t\n\x0b\x0c\r")
    for f in range(100):
        if off[f + 1] > off[f]:
            assert t[off[f + 1] - 1] in ws  # every file ends in whitespace (separator contract)


def test_shard_equals_slices_of_the_corpus():
    # a GPU's shard (bench.py strong scaling) is byte-identical to its files' slices of the whole corpus
    t, off = ii_ctypes.zipf_corpus(2_000_000, 53, 3000, 11, threads=3)
    assert (ii_ctypes.zipf_layout(2_000_000, 53, 11) == off).all()
    sizes = [int(off[i + 1] - off[i]) for i in range(53)]
    order, sb, se = ii_ctypes.partition(sizes, 4)
    for g in range(4):
        files = sorted(order[sb[g]:se[g]])
        s, so = ii_ctypes.zipf_shard(2_000_000, 53, 3000, 11, files, threads=2)
        exp = b"".join(t[int(off[f]):int(off[f + 1])].tobytes() for f in files)
        assert s.tobytes() == exp
        assert [int(x) for x in so[1:] - so[:-1]] == [sizes[f] for f in files]
    s, so = ii_ctypes.zipf_shard(2_000_000, 53, 3000, 11, [], threads=2)
    assert len(s) == 0 and list(so) == [0]


def test_golden_zipf_corpus_reproduces():
    import json, os
    from conftest import GOLDEN
    meta = json.load(open(os.path.join(GOLDEN, "golden.json")))["cases"]["zipf_small"]["iigen"]
    t, _ = ii_ctypes.zipf_corpus(meta["total_bytes"], meta["nfiles"], meta["vocab"], meta["seed"], threads=3)
    assert hashlib.sha256(t.tobytes()).hexdigest() == meta["corpus_sha256"]
