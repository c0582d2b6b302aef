"""CPU: the oracle (C restatement, oracle/ii_oracle.c) is pinned against the
reference binary's own outputs (tests/golden/, made by make_golden.py)."""
import hashlib
import json
import os
import subprocess
import tempfile

import pytest

from conftest import CASES, GOLDEN, ORACLE, case_arrays, load_case, materialize, partials_meta, size_order
from oracle_py import oracle_index, oracle_partials


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference_goldens(case):
    text, off, ids, expected = case_arrays(case)
    got = oracle_index(text, off, ids)
    for l in "abcdefghijklmnopqrstuvwxyz":
        assert got[l] == expected[l], "letter %s differs" % l


@pytest.mark.parametrize("threads", [2, 3, 8, 40])
@pytest.mark.parametrize("case", ["config1", "config2", "edge", "rand_1", "tiny360", "zipf_small"])
def test_multithreaded_oracle_matches_reference_goldens(case, threads):
    # the full-size CPU baseline of bench.py (ii_oracle_index_mt), incl. more threads than files
    text, off, ids, expected = case_arrays(case)
    got = oracle_index(text, off, ids, threads=threads)
    for l in "abcdefghijklmnopqrstuvwxyz":
        assert got[l] == expected[l], "letter %s differs" % l


def test_multithreaded_oracle_matches_single_thread_zipf():
    import ii_ctypes
    t, off = ii_ctypes.zipf_corpus(30_000_000, 500, 300_000, 4, threads=8)
    ids = [2 * i + 1 for i in range(500)]
    assert oracle_index(t, off, ids, threads=7) == oracle_index(t, off, ids)


def test_golden_json_consistent():
    meta = json.load(open(os.path.join(GOLDEN, "golden.json")))
    # config 1 / config 2 aggregate hashes of the reference
    assert meta["cases"]["config1"]["sha256"].startswith("8968c9ae0ce82a20")
    assert meta["cases"]["config2"]["sha256"].startswith("47a8ad1e4b6f28c3")
    assert meta["cases"]["config2"]["lines"] == 33262
    assert meta["cases"]["config2"]["out_bytes"] == 1380621
    for case in CASES:
        _, _, _, expected = case_arrays(case)
        allb = b"".join(expected[l] for l in "abcdefghijklmnopqrstuvwxyz")
        assert hashlib.sha256(allb).hexdigest() == meta["cases"][case]["sha256"]


@pytest.mark.parametrize("case", ["config1", "edge", "tiny360"])
def test_oracle_cli_matches(case):
    with tempfile.TemporaryDirectory() as td:
        _, _, expected = materialize(case, td)
        subprocess.run([os.path.join(ORACLE, "build", "ii_oracle"), "2", "3", "list.txt"], cwd=td, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        for l in "abcdefghijklmnopqrstuvwxyz":
            assert open(os.path.join(td, l + ".txt"), "rb").read() == expected[l]


def test_oracle_defined_ub_long_token():
    # raw token >= 300 bytes: reference UB (stack overflow); defined as keeping
    # the first 299 letters
    text = b"A" * 500 + b" b"
    got = oracle_index(text, [0, len(text)], [0])
    assert got["a"] == b"a" * 299 + b":[1]\n"
    assert got["b"] == b"b:[1]\n"


@pytest.mark.parametrize("case", CASES)
def test_oracle_partials_match_reference(case):
    # the reference's partial_<l>.txt with M = 1 (tests/golden/make_partial_golden.py)
    text, off, ids, _ = case_arrays(case)
    got = oracle_partials(text, off, ids, size_order(case))
    meta = partials_meta()[case]
    for l in "abcdefghijklmnopqrstuvwxyz":
        assert hashlib.sha256(got[l]).hexdigest() == meta[l]["sha256"], "partial_%s.txt differs" % l


def test_partition_order_is_size_order():
    import ii_ctypes
    for case in CASES:
        list_text, files, _ = load_case(case)
        toks = list_text.split()
        paths = toks[1:1 + int(toks[0])]
        sizes = [len(files[p]) if p in files else 0 for p in paths]
        order, sb, se = ii_ctypes.partition(sizes, 1)
        assert order == size_order(case) and (sb[0], se[0]) == (0, len(paths))


def test_streaming_oracle_matches_whole_corpus():
    """The streaming, letter-range oracle (configs[4]'s hashes) gives the
    whole-corpus oracle's letters: files in 4 ascending-id batches, the
    letters in three passes of ranges."""
    import hashlib
    import ii_ctypes
    from oracle_py import OracleStream, oracle_index
    t, off = ii_ctypes.zipf_corpus(3_000_000, 57, 40_000, 9, threads=4)
    off = [int(x) for x in off]
    ids = [3 * f + 1 for f in range(57)]  # ascending, not dense
    exp = oracle_index(t, off, ids)
    cuts = [0, 5, 23, 40, 57]
    for lo, hi in [(0, 9), (9, 10), (10, 26)]:
        st = OracleStream(lo, hi)
        for a, b in zip(cuts, cuts[1:]):
            st.add(t[off[a]:off[b]], [o - off[a] for o in off[a:b + 1]], ids[a:b], threads=3)
        for l in range(lo, hi):
            h = hashlib.sha256()
            nbytes, lines = st.letter(l, h.update)
            e = exp[chr(97 + l)]
            assert (h.hexdigest(), nbytes, lines) == (hashlib.sha256(e).hexdigest(), len(e), e.count(b"\n"))
        st.close()
