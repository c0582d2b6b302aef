#!/usr/bin/env python3
"""Phase timing of the N > 1 path on ONE GPU (timing experiment, not product
code): G logical shards of a Zipf corpus, each mapped in its own context on
cuda:0 (rank-contiguous files, as bench.py lays them out), then the same
steps ii_dist.exchange_and_reduce runs per rank — local reduce, plan +
export, the exchange (device copies here; RCCL all-to-allv on a node),
import, order + format — each timed across all G contexts.

    python tools/exchange_timing.py [bytes_per_shard] [G] [steps] [interleaved] [corpus]

interleaved = 1: shard g owns files g, g + G, g + 2G, ... (the id ranges of
the sources overlap, as with bench.py's ii_partition shards, so the owners
sort their merged pairs instead of merging ordered runs).
owner_ms_*: the owners' device time per ii_import phase (hipEvents inside
libii: word tokenisation, dictionary, merge / sort, unique) and order / format.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "bindings"))

import torch  # noqa: E402

import ii_ctypes  # noqa: E402
import ii_dist  # noqa: E402


def main():
    nb = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(2e9)
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    inter = len(sys.argv) > 4 and sys.argv[4] == "1"
    # corpus (5th argument): the G shards are ii_partition's shares of ONE corpus of G * bytes_per_shard
    # (as bench.py --gpus G lays them out: one vocabulary, size-sorted files, interleaved ids);
    # otherwise every shard is a corpus of its own (its own seed, so its own words)
    one = len(sys.argv) > 5 and sys.argv[5] == "corpus"
    files = 2000
    texts = []
    if one:
        layout = ii_ctypes.zipf_layout(nb * G, files * G, 3)
        order, sb, se = ii_ctypes.partition([int(x) for x in (layout[1:] - layout[:-1])], G)
    for g in range(G):
        if one:
            ids = sorted(order[sb[g]:se[g]])
            t, off = ii_ctypes.zipf_shard(nb * G, files * G, 1_000_000, 3, ids, threads=16)
        else:
            t, off = ii_ctypes.zipf_corpus(nb, files, 1_000_000, 3 + 1000 * g, threads=16)
            ids = list(range(g, G * files, G)) if inter else list(range(g * files, (g + 1) * files))
        n = int(off[-1])
        d = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        d[:n].copy_(torch.from_numpy(t[:n]))
        texts.append((d, off[:-1].tolist(), ids, n))
    torch.cuda.synchronize()
    idxs = [ii_ctypes.Index(0) for _ in range(G)]
    res = []
    for it in range(steps + 1):
        ph = {}

        def lap(name, t0):
            torch.cuda.synchronize()
            ph[name] = ph.get(name, 0.0) + (time.perf_counter() - t0) * 1e3

        for g, ix in enumerate(idxs):
            t0 = time.perf_counter()
            d, fs, ids, n = texts[g]
            ix.map_device(d.data_ptr(), n, fs, ids)
            lap("map", t0)
            t0 = time.perf_counter()
            ix.reduce_local()
            lap("reduce_local", t0)
        t0 = time.perf_counter()
        lo, hi = ii_dist.owner_ranges([ix.letter_load() for ix in idxs], G)
        sends = []
        for ix in idxs:
            sizes = ix.export_plan_ranges(lo, hi)
            off, total = ii_dist.prefix(sizes)
            buf = torch.empty(max(total, 8), dtype=torch.uint8, device="cuda")
            ix.export(G, buf.data_ptr(), off)
            sends.append((buf, sizes, off))
        lap("plan_export", t0)
        recvs = []
        t0 = time.perf_counter()
        for dst in range(G):
            parts = [s[0][s[2][dst]:s[2][dst] + s[1][dst]] for s in sends]
            recv_sizes = [s[1][dst] for s in sends]
            recvs.append((torch.cat(parts) if sum(recv_sizes) else torch.empty(8, dtype=torch.uint8, device="cuda"),
                          recv_sizes))
        lap("exchange_copies", t0)
        for dst, ix in enumerate(idxs):
            t0 = time.perf_counter()
            recv, rs = recvs[dst]
            ix.import_(G, recv.data_ptr(), ii_dist.prefix(rs)[0], G * files)
            lap("import", t0)
            t0 = time.perf_counter()
            ix.reduce(copy_text=False)
            lap("order_format", t0)
            # the owner's device-side phases of ii_import (+ order / format): events inside libii
            st = ix.stats()
            for k in ("ms_map", "ms_dict", "ms_sort", "ms_reduce", "ms_order", "ms_format"):
                ph["owner_" + k] = ph.get("owner_" + k, 0.0) + getattr(st, k)
        ph["exchange_bytes"] = sum(sum(s[1]) for s in sends)
        if it:
            res.append(ph)
    avg = {k: round(sum(r[k] for r in res) / len(res), 2) for k in res[0]}
    avg["per_shard_ms"] = {k: round(v / G, 3) for k, v in avg.items() if k != "exchange_bytes"}
    print(json.dumps({"G": G, "bytes_per_shard": nb, "interleaved_ids": inter or one, "one_corpus": one, "id_sort": bool(os.environ.get("II_IMPORT_ID_SORT")),
                      "phases_ms_all_shards": avg}))
    for ix in idxs:
        ix.close()


if __name__ == "__main__":
    main()
