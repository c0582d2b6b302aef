"""GPU: the benchmark corpora at FULL size against the oracle — every letter
of the index of BASELINE configs[2] (10 GB, 10^4 files, vocab 10^6, seed 3),
of a configs[4]-sized corpus (12.5 GB, 1.25*10^5 files, vocab 10^7, seed 5)
and of rank 0's ii_partition share of configs[4] over 8 GPUs, hashed and compared with tests/golden/bench_hashes.json (made by the
oracle in the build container, tests/golden/make_bench_hashes.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

import ii_ctypes
from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DB = json.load(open(os.path.join(GOLDEN, "bench_hashes.json")))["workloads"]


def share_ids(p, rank, world):
    """Global ids of the files ii_partition (main.c:300-323, M = world) gives shard `rank`."""
    layout = ii_ctypes.zipf_layout(p["total_bytes"], p["nfiles"], p["seed"])
    order, sb, se = ii_ctypes.partition([int(x) for x in (layout[1:] - layout[:-1])], world)
    return sorted(order[sb[rank]:se[rank]])


@pytest.mark.parametrize("name", ["config3", "config5share", "config5/share0of8", "config5/share7of8"])
def test_full_size_index_matches_oracle(name):
    """config5/share<r>of8: rank r's ii_partition share of configs[4] over 8
    GPUs (main.c:300-323 with M = 8), with the files' GLOBAL ids in [0, 10^6)
    — the shape a real rank indexes.  Rank 0 holds the 15 835 largest files
    (14-bit shard-local file indices), rank 7 the 439 993 smallest (19-bit
    indices: the widest sort keys of the job)."""
    import torch
    if name not in DB:
        pytest.skip("no oracle hashes for %s" % name)
    w = DB[name]
    p = w["iigen"]
    _, _, share = name.partition("/")
    if share:
        r, g = (int(x) for x in share[len("share"):].split("of"))
        ids = share_ids(p, r, g)
        text, off = ii_ctypes.zipf_shard(p["total_bytes"], p["nfiles"], p["vocab"], p["seed"], ids, threads=16)
    else:
        ids = list(range(p["nfiles"]))
        text, off = ii_ctypes.zipf_corpus(p["total_bytes"], p["nfiles"], p["vocab"], p["seed"], threads=16)
    n = int(off[-1])
    d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    d[:n].copy_(torch.from_numpy(text))
    torch.cuda.synchronize()
    del text
    with ii_ctypes.Index(0) as ix:
        ix.map_device(d.data_ptr(), n, off[:-1].tolist(), ids)
        ix.reduce(copy_text=True)
        st = ix.stats()
        assert st.words == w["words"] and st.out_bytes == w["out_bytes"]
        bad = [l for l in w["letters"] if hashlib.sha256(ix.letter_text(ord(l) - 97)).hexdigest()
               != w["letters"][l]["sha256"]]
        if share:
            assert st.sort_packed == 1
    assert not bad, "letters differ from the oracle: %s" % bad


@pytest.mark.parametrize("G", [2, 4, 8])
def test_logical_shards_full_size(G):
    """BASELINE configs[3] at full size through the sharded path on one GPU:
    the 10 GB config3 corpus cut by ii_partition (main.c:300-323, M = G) into
    G contexts, each mapping and locally reducing its share with the files'
    global ids; every context exports its letter segments, the owner of
    ii_reducer_letters(r, G) (main.c:129-130) imports the G segments (the
    merge-path owner merge, ~5*10^7 records per owner at G = 8) and formats
    its letters.  The letters of all owners together must hash like the
    oracle's index of the whole corpus (tests/golden/bench_hashes.json)."""
    import torch
    import ii_dist
    w = DB["config3"]
    p = w["iigen"]
    idxs, bufs = [], []
    try:
        for g in range(G):
            ids = share_ids(p, g, G)
            text, off = ii_ctypes.zipf_shard(p["total_bytes"], p["nfiles"], p["vocab"], p["seed"], ids, threads=16)
            n = int(off[-1])
            d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
            d[:n].copy_(torch.from_numpy(text))
            torch.cuda.synchronize()
            del text
            ix = ii_ctypes.Index(0)
            idxs.append(ix)
            bufs.append(d)
            ix.map_device(d.data_ptr(), n, off[:-1].tolist(), ids)
        los, his = ii_dist.logical_shards_reduce(idxs, p["nfiles"], copy_text=True)
        got, words, out_bytes = {}, 0, 0
        for g, ix in enumerate(idxs):
            assert (los[g], his[g]) == ii_ctypes.reducer_letters(g, G)
            for l in range(26):
                t = ix.letter_text(l)
                if los[g] <= l < his[g]:
                    got[chr(97 + l)] = hashlib.sha256(t).hexdigest()
                    words += t.count(b"\n")
                    out_bytes += len(t)
                else:
                    assert t == b"", "owner %d holds letter %s it does not own" % (g, chr(97 + l))
        assert words == w["words"] and out_bytes == w["out_bytes"]
        bad = [l for l in w["letters"] if got.get(l) != w["letters"][l]["sha256"]]
        assert not bad, "G=%d: letters differ from the oracle: %s" % (G, bad)
    finally:
        for ix in idxs:
            ix.close()
