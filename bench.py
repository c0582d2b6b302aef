#!/usr/bin/env python3
"""Benchmark: indexed input GB/s of the MI355X inverted-index builder.

Workload (BASELINE.json configs[2]): synthetic Zipf corpus,
10 GB across 10^4 files, vocabulary 10^6, seed 3, one MI355X per rank.  A
"step" is one full pass of the hot path over the corpus: tokenize (K1), word
table + lexicographic ids, token sort (K2), unique pairs (K3), final order
(K4) and the formatted a..z index text (K5), all device-resident — the text
is already in HBM when the timed region starts; nothing is cached across
steps (every step re-tokenizes and rebuilds the index from scratch).

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1 is launched by torch.distributed.run (one process per GPU).  Each rank
indexes its own 10 GB corpus (weak scaling): map + local reduce on its shard,
one RCCL all-to-allv of letter ranges (ii_dist.exchange_and_reduce), and the
owner's merge + order + format.  Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "parallel-computation-of-an-inverted-index-using-map-reduce_amd")
sys.path.insert(0, os.path.join(PKG, "bindings"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--bytes", type=float, default=10e9, help="corpus bytes per rank")
    p.add_argument("--files", type=int, default=10_000)
    p.add_argument("--vocab", type=int, default=1_000_000)
    p.add_argument("--seed", type=int, default=3)
    p.add_argument("--cpu-sample-bytes", type=float, default=48e6)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--gen-threads", type=int, default=16)
    p.add_argument("--io-bytes", type=float, default=2e9,
                   help="bytes of the corpus written to files for the ii_map_files reader leg (0 = skip)")
    p.add_argument("--letter-split", choices=["balanced", "reference"], default="balanced",
                   help="letter ownership of the N>1 exchange: histogram-balanced (SURVEY §8 f4) or the "
                        "reference's 26/N reducer split (main.c:129-130)")
    return p.parse_args()


def pmc_traffic():
    """HBM bytes per launch by kernel from the committed rocprofv3 PMC summary
    of this same bench command (profiles/*_pmc_traffic.json, newest round),
    corrected as profiles/pmc_traffic.py documents; {} when absent."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")))
    if not files:
        return {}
    try:
        d = json.load(open(files[-1]))
        return {k: round(v["traffic_bytes_per_launch"]) for k, v in d["kernels"].items()
                if "traffic_bytes_per_launch" in v}
    except Exception:
        return {}


def safe_mappers(sizes, cores):
    """Largest M <= cores for which the reference's greedy split (main.c:307-323)
    initialises every mapper's range; with more mappers than realised shards
    the reference reads uninitialised file_start/end and crashes."""
    order = sorted(sizes, reverse=True)
    total = sum(sizes)
    for M in range(cores, 0, -1):
        per, cur, cum = total // M, 0, 0
        for s in order:
            cum += s
            if cum >= per and cur < M - 1:
                cur, cum = cur + 1, 0
        if cur == M - 1:
            return M
    return 1


def cpu_baseline(text, off, sample_bytes):
    """Time the reference itself (oracle/_ref/tema1, gcc -O2 build of
    /root/reference/main.c) on the first files of the same corpus."""
    import numpy as np
    ref = os.path.join(REPO, "oracle", "_ref", "tema1")
    nf = 0
    while nf < min(360, len(off) - 1) and off[nf + 1] <= sample_bytes:  # reference MAX_FILES = 360
        nf += 1
    nf = max(nf, 1)
    sb = int(off[nf])
    cores = safe_mappers([int(off[f + 1] - off[f]) for f in range(nf)], min(16, os.cpu_count() or 1))
    sample = "first %d files of the corpus (%.1f MB), M=%d mappers, R=26 reducers" % (nf, sb / 1e6, cores)
    if os.path.exists(ref):
        td = tempfile.mkdtemp(prefix="ii_cpu_")
        try:
            names = []
            for f in range(nf):
                p = os.path.join(td, "f%05d.txt" % f)
                np.asarray(text[int(off[f]):int(off[f + 1])]).tofile(p)
                names.append(p)
            with open(os.path.join(td, "list.txt"), "w") as fl:
                fl.write("%d\n%s\n" % (nf, "\n".join(names)))
            t0 = time.perf_counter()
            subprocess.run([ref, str(cores), "26", "list.txt"], cwd=td, check=True, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL, timeout=600)
            dt = time.perf_counter() - t0
        finally:
            shutil.rmtree(td, ignore_errors=True)
        return {"value": round(sb / dt / 1e9, 6), "unit": "GB/s", "cores": cores, "kind": "reference",
                "sample": sample, "seconds": round(dt, 3)}
    # reference binary absent: the oracle restatement, single thread
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_py import oracle_index
    t0 = time.perf_counter()
    oracle_index(text[:sb], off[:nf + 1], list(range(nf)))
    dt = time.perf_counter() - t0
    return {"value": round(sb / dt / 1e9, 6), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": sample.replace("M=%d mappers, R=26 reducers" % cores, "oracle restatement, 1 thread"),
            "seconds": round(dt, 3)}


def io_leg(idx, text, off, io_bytes, threads=16):
    """End-to-end file leg, reported beside `value`, never as
    it: the first files of the corpus (<= io_bytes) are written to a scratch
    directory, then ii_map_files reads them (pipelined pread into pinned
    windows + async H2D, `threads` readers) and maps them.  Page cache warm
    (the files were just written); best of 2."""
    import numpy as np
    nf = 0
    while nf < len(off) - 1 and off[nf + 1] <= io_bytes:
        nf += 1
    if nf == 0:
        return None
    td = tempfile.mkdtemp(prefix="ii_io_")
    try:
        paths = []
        for f in range(nf):
            p = os.path.join(td, "f%05d.txt" % f)
            np.asarray(text[int(off[f]):int(off[f + 1])]).tofile(p)
            paths.append(p)
        best = None
        for _ in range(2):
            t0 = time.perf_counter()
            idx.map_files(paths, nthreads=threads)
            wall = time.perf_counter() - t0
            st = idx.stats()
            if best is None or wall < best[0]:
                best = (wall, st.io_ms, st.io_bytes, st.ms_map)
    finally:
        shutil.rmtree(td, ignore_errors=True)
    wall, io_ms, io_b, map_ms = best
    return {"files": nf, "bytes": int(off[nf]), "threads": threads, "read_upload_ms": round(io_ms, 2),
            "read_upload_GBps": round(io_b / (io_ms * 1e-3) / 1e9, 2) if io_ms > 0 else None,
            "map_files_ms": round(wall * 1e3, 2), "map_files_GBps": round(int(off[nf]) / wall / 1e9, 2),
            "k1_ms": round(map_ms, 2), "page_cache": "warm"}


def main():
    a = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    import ii_ctypes
    import ii_dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one process per GPU over RCCL (backend "nccl"); II_DIST_BACKEND=gloo rehearses the N>1 path on
        # fewer GPUs (ranks share devices, collectives go through host memory) — never for measurements
        backend = os.environ.get("II_DIST_BACKEND", "nccl")
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)

    # ---- corpus: this rank's 10 GB (seed differs per rank), then to HBM
    nbytes = int(a.bytes)
    t0 = time.perf_counter()
    text, off = ii_ctypes.zipf_corpus(nbytes, a.files, a.vocab, a.seed + 1000 * rank, threads=a.gen_threads)
    gen_s = time.perf_counter() - t0
    d_text = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
    d_text[:nbytes].copy_(torch.from_numpy(text))
    torch.cuda.synchronize()
    file_start = off[:-1].tolist()
    # global file IDs: rank r owns files [r*F, (r+1)*F)
    ids = list(range(rank * a.files, (rank + 1) * a.files))

    idx = ii_ctypes.Index(local if world > 1 else 0)

    id_bound = world * a.files

    def step():
        idx.map_device(d_text.data_ptr(), nbytes, file_start, ids)
        if world > 1:  # local reduce -> letter-range all-to-allv (RCCL) -> owner merge + format
            ii_dist.exchange_and_reduce(idx, id_bound, balanced=a.letter_split == "balanced")
        else:
            idx.reduce(copy_text=False)

    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scatter_ms, emit_ms, phase_ms = [], [], []
    for _ in range(a.steps):
        step()
        st = idx.stats()
        scatter_ms.append(st.scatter_ms_avg)
        emit_ms.append(st.emit_ms)
        phase_ms.append(st.ms_sort + st.ms_reduce)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    st = idx.stats()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / a.steps * 1e3
    total_bytes = nbytes * world
    value = total_bytes * a.steps / dt / 1e9

    if rank == 0:
        sc_ms = sum(scatter_ms) / len(scatter_ms)
        sc_achieved = st.scatter_bytes / (sc_ms * 1e-3) / 1e9 if sc_ms > 0 else 0.0
        em_ms = sum(emit_ms) / len(emit_ms)
        em_achieved = st.emit_bytes / (em_ms * 1e-3) / 1e9 if em_ms > 0 else 0.0
        traffic = pmc_traffic()
        # sort + segmented-reduce phase (K2 token sort + K3 unique), SURVEY §8d byte model:
        # first pass 8 B per record read + 8 B per kept record written; each scatter pass
        # 16 B per kept record; each later histogram pass 8 B per kept record; the unique
        # scan reads the kept records twice and writes 16 B (pair + posting offset) per pair
        T, Tk, U = st.tokens, st.sorted_records, st.pairs
        sp = max(1, st.sort_passes)
        ph_bytes = 8 * T + 8 * Tk + sp * 16 * Tk + (sp - 1) * 8 * Tk + 2 * 8 * Tk + 16 * U
        ph_ms = sum(phase_ms) / len(phase_ms)
        ph_achieved = ph_bytes / (ph_ms * 1e-3) / 1e9 if ph_ms > 0 else 0.0
        cpu = None if a.no_cpu_baseline or world > 1 else cpu_baseline(text, off, a.cpu_sample_bytes)
        io = io_leg(idx, text, off, a.io_bytes) if world == 1 and a.io_bytes > 0 else None
        line = {
            "metric": "indexed input GB/s (whole node) + % of HBM peak BW",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic Zipf corpus (tools/iigen.c, s~1, seed %d+1000*rank), device-resident" % a.seed,
            "config": {"workload": "zipf %.3g GB x %d files/rank, vocab %d (BASELINE configs[2])" % (
                nbytes / 1e9, a.files, a.vocab), "bytes_per_rank": nbytes, "files_per_rank": a.files,
                "vocab": a.vocab, "parallelism": "shard-per-gpu x%d" % world,
                "letter_split": a.letter_split if world > 1 else None},
            # dominant kernel: the tokenizer (K1b); algorithmic bytes = B + 8*T per launch
            "roofline": {"bound": "hbm", "kernel": "k_tok_emit (K1b tokenizer)",
                         "achieved": round(em_achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(em_achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic.get("ii::k_tok_emit<0>"),
                         "bytes_per_launch": st.emit_bytes, "ms_per_launch": round(em_ms, 4)},
            "roofline_sort": {"bound": "hbm", "kernel": "k_radix_scatter (token sort passes)",
                              "achieved": round(sc_achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(sc_achieved / HBM_PEAK_GBS, 4),
                              "bytes_per_launch": st.scatter_bytes, "ms_per_launch": round(sc_ms, 4)},
            "roofline_sort_phase": {"bound": "hbm", "phase": "token sort + segmented unique (K2 + K3)",
                                    "achieved": round(ph_achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": round(ph_achieved / HBM_PEAK_GBS, 4), "bytes_per_step": ph_bytes,
                                    "ms_per_step": round(ph_ms, 4),
                                    "first_pass": {"kernel": "k_sort0_compact", "ms": round(st.sort0_ms, 4),
                                                   "bytes": st.sort0_bytes,
                                                   "achieved": round(st.sort0_bytes / (st.sort0_ms * 1e-3) / 1e9, 1)
                                                   if st.sort0_ms > 0 else 0.0}},
            "cpu_baseline": cpu,
            "io": io,
            "phases_ms": {k: round(getattr(st, k), 3) for k in
                          ["ms_map", "ms_dict", "ms_sort", "ms_reduce", "ms_order", "ms_format", "ms_total",
                           "emit_ms", "resolve_ms"]},
            "counts": {"tokens": st.tokens, "pairs": st.pairs, "words": st.words, "long_tokens": st.long_tokens,
                       "out_bytes": st.out_bytes, "sort_passes": st.sort_passes, "table_cap": st.table_cap,
                       "resolved_tokens": st.resolved_tokens, "sorted_records": st.sorted_records},
            "gen_seconds": round(gen_s, 2),
        }
        print(json.dumps(line), flush=True)
    idx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
