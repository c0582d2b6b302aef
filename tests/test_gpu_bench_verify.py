"""GPU: the benchmark corpora at FULL size against the oracle — every letter
of the index of BASELINE configs[2] (10 GB, 10^4 files, vocab 10^6, seed 3),
of a configs[4]-sized corpus (12.5 GB, 1.25*10^5 files, vocab 10^7, seed 5)
and of rank 0's ii_partition share of configs[4] over 8 GPUs, hashed and compared with tests/golden/bench_hashes.json (made by the
oracle in the build container, tests/golden/make_bench_hashes.py)."""
import hashlib
import json
import os
import sys
import time

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


@pytest.mark.parametrize("name,G", [("config3", 2), ("config3", 4), ("config3", 8), ("config5share", 8)])
def test_logical_shards_full_size(name, G):
    """BASELINE configs[3] at full size through the sharded path on one GPU:
    the 10 GB config3 corpus cut by ii_partition (main.c:300-323, M = G) into
    G contexts, each mapping and locally reducing its share with the files'
    global ids; every context exports its letter segments, the owner of
    ii_reducer_letters(r, G) (main.c:129-130) imports the G segments (the
    merge-path owner merge, ~5*10^7 records per owner at G = 8) and formats
    its letters.  The letters of all owners together must hash like the
    oracle's index of the whole corpus (tests/golden/bench_hashes.json).
    config5share: configs[4]'s generator at one GPU's share of its size
    (12.5 GB, 1.25*10^5 files, vocabulary 10^7, seed 5) through the same
    G = 8 exchange — every owner merges 8 segments of ~10^6-10^7-word
    dictionaries with 17-bit ids, the segmented-reduce stress of configs[4]."""
    import torch
    import ii_dist
    w = DB[name]
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
        assert not bad, "%s G=%d: letters differ from the oracle: %s" % (name, G, bad)
    finally:
        for ix in idxs:
            ix.close()


# BASELINE configs[4]: 100 GB over 10^6 files, vocabulary 10^7 (bench.py --workload config5)
CONFIG5 = {"total_bytes": 100_000_000_000, "nfiles": 1_000_000, "vocab": 10_000_000, "seed": 5}


def _progress(msg):
    # (run with -s on the GPU box: a line every share / owner, so a long test is not taken for a hang)
    sys.stdout.write("[config5 %.0fs] %s\n" % (time.time() - _progress.t0, msg))
    sys.stdout.flush()


@pytest.mark.timeout(1500)
def test_config5_full_exchange():
    """BASELINE configs[4] at its FULL size through the exchange, on one GPU in
    sequence — what an 8-GPU job does, one rank and one owner at a time:
      * each of the 8 ii_partition shares (main.c:300-323 with M = 8: 12.5 GB,
        15 835 ... 439 993 files, their GLOBAL ids in [0, 10^6)) is generated,
        mapped, locally reduced and exported into a device send buffer (the
        segments for all 8 owners), and its context closed;
      * each owner r (letters ii_reducer_letters(r, 8), main.c:129-130) then
        imports its 8 segments (20-bit ids, dictionaries of ~10^6 words, the
        merge-path owner merge of ~10^9 pairs), orders and formats its letters.
    No oracle output exists at this size; every letter file is checked for the
    properties the reference's writer guarantees (oracle/ii_check.c: line
    syntax, ids strictly ascending in [1, 10^6], (df desc, word asc) order,
    the file's first letter), each owner holds only its letters, and per letter
    the sum of df over the output equals the sum of the 8 shares' distinct
    (word, file) pairs of that letter (files are disjoint across shares, so
    local pairs add up to global ones).  With oracle hashes for the corpus in
    tests/golden/bench_hashes.json ("config5") the letters must match them."""
    import torch
    from index_check import KINDS, check_letter
    import ii_dist
    _progress.t0 = time.time()
    p = CONFIG5
    G = 8
    layout = ii_ctypes.zipf_layout(p["total_bytes"], p["nfiles"], p["seed"])
    order, sb, se = ii_ctypes.partition([int(x) for x in (layout[1:] - layout[:-1])], G)
    del layout
    lo, hi = zip(*[ii_ctypes.reducer_letters(r, G) for r in range(G)])
    lo, hi = list(lo), list(hi)
    sends, load, share_pairs, share_words = [], [0] * 26, 0, []
    for g in range(G):
        ids = sorted(order[sb[g]:se[g]])
        text, off = ii_ctypes.zipf_shard(p["total_bytes"], p["nfiles"], p["vocab"], p["seed"], ids, threads=16)
        n = int(off[-1])
        d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        d[:n].copy_(torch.from_numpy(text))
        torch.cuda.synchronize()
        del text
        with ii_ctypes.Index(0) as ix:
            ix.map_device(d.data_ptr(), n, off[:-1].tolist(), ids)
            ix.reduce_local()
            ld = ix.letter_load()
            st = ix.stats()
            sizes = ix.export_plan_ranges(lo, hi)
            soff, total = ii_dist.prefix(sizes)
            buf = torch.empty(max(total, 8), dtype=torch.uint8, device="cuda")
            ix.export(G, buf.data_ptr(), soff)
        torch.cuda.synchronize()
        del d
        torch.cuda.empty_cache()
        assert st.pairs == sum(ld) and st.bytes == n
        load = [a + b for a, b in zip(load, ld)]
        share_pairs += st.pairs
        share_words.append(st.words)
        sends.append((buf, sizes, soff))
        _progress("share %d: %d files, %.2f GB, %d tokens, %d words, %d pairs, %.2f GB of segments"
                  % (g, len(ids), n / 1e9, st.tokens, st.words, st.pairs, total / 1e9))
    ref = DB.get("config5")
    words = pairs = out_bytes = 0
    bad_hash = []
    for r in range(G):
        parts = [s[0][s[2][r]:s[2][r] + s[1][r]] for s in sends]
        recv_sizes = [s[1][r] for s in sends]
        recv = torch.cat(parts)
        torch.cuda.synchronize()
        with ii_ctypes.Index(0) as ix:
            ix.import_(G, recv.data_ptr(), ii_dist.prefix(recv_sizes)[0], p["nfiles"])
            ix.reduce(copy_text=True)
            st = ix.stats()
            lines = sdf = nbytes = 0
            for l in range(26):
                t = ix.letter_text(l)
                if not lo[r] <= l < hi[r]:
                    assert t == b"", "owner %d holds letter %s it does not own" % (r, chr(97 + l))
                    continue
                rc, nl, s_df, mdf, at = check_letter(t, l, p["nfiles"], 16)
                assert rc == 0, "letter %s: %s at byte %d: %r" % (chr(97 + l), KINDS.get(rc, rc), at,
                                                                   t[max(0, at - 60):at + 60])
                assert s_df == load[l], "letter %s: sum of df %d, shares' pairs %d" % (chr(97 + l), s_df, load[l])
                lines += nl
                sdf += s_df
                nbytes += len(t)
                if ref and hashlib.sha256(t).hexdigest() != ref["letters"][chr(97 + l)]["sha256"]:
                    bad_hash.append(chr(97 + l))
                del t
            assert st.words == lines and st.pairs == sdf and st.out_bytes == nbytes
        del recv, parts
        torch.cuda.empty_cache()
        words += lines
        pairs += sdf
        out_bytes += nbytes
        _progress("owner %d (letters %s-%s): %d words, %d pairs, %.2f GB of text, checked"
                  % (r, chr(97 + lo[r]), chr(96 + hi[r]), lines, sdf, nbytes / 1e9))
    assert pairs == share_pairs
    # the whole vocabulary holds at least any one share's words and at most the generator's vocabulary
    assert max(share_words) <= words <= p["vocab"]
    if ref:
        assert words == ref["words"] and out_bytes == ref["out_bytes"]
        assert not bad_hash, "letters differ from the oracle: %s" % bad_hash
