#!/usr/bin/env python3
"""Benchmark: indexed input GB/s of the MI355X inverted-index builder.

Workloads (BASELINE.json configs):
  config3       synthetic Zipf corpus, 10 GB across 10^4 files, vocabulary 10^6,
                seed 3 — configs[2] on one MI355X; configs[3] ("the same corpus
                sharded over 2/4/8") for N > 1
  config5       BASELINE configs[4]: 100 GB across 10^6 files, vocabulary 10^7,
                seed 5 — the named --gpus 8 run (strong scaling: every rank
                generates and indexes its ii_partition share); on one GPU only
                as --rank-share r/N
  config5share  a configs[4]-sized single-GPU corpus: 12.5 GB across
                1.25*10^5 files, vocabulary 10^7, seed 5 (ids 0 .. 1.25*10^5)
A "step" is one full pass of the hot path over the corpus: tokenize (K1), word
table + lexicographic ids, token sort (K2), unique pairs (K3), final order
(K4) and the formatted a..z index text (K5), all device-resident — the text
is already in HBM when the timed region starts; nothing is cached across
steps (every step re-tokenizes and rebuilds the index from scratch).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config3|config5|config5share]
                    [--scaling strong|weak] [--rank-share r/N] [--letter-split reference|balanced]

--rank-share r/N (one GPU): the share of rank r when the workload is strong-
scaled over N GPUs — the files ii_partition (M = N, main.c:300-323) gives
shard r, generated with their GLOBAL ids (for configs[4] at N = 8: 1.25*10^5
files whose ids span [0, 10^6)); a step maps and reduces that share (the full
local index, as at N = 1), and an `export` leg times what the rank does before
the exchange (map + local reduce + ii_export_plan + ii_export).  Verified
against the oracle's hashes of that share (tests/golden/bench_hashes.json).

--gpus N > 1 without a torch.distributed environment starts
`python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child
(before anything touches a GPU) and exits with its return code; one process
per GPU, RCCL (backend "nccl") for the exchange.  Strong scaling (default):
the files of the ONE corpus are assigned to ranks by the reference's size
heuristic (ii_partition with M = N, main.c:300-323); each rank generates only
its own files, maps and locally reduces them, one all-to-allv routes each
letter range to its owner (by default the reference's reducer split with
R = N, main.c:129-130, as north_star asks; --letter-split balanced: the
histogram-balanced ranges of SURVEY §8 f4), and the owners merge and format.
--scaling weak: every rank indexes its own full-size corpus (seed + 1000*rank).

After the timed loop (outside it) one more step copies the text out and every
letter's sha256 is compared with tests/golden/bench_hashes.json (made by the
oracle in the build container): "verified" in the JSON line.  Rank 0 prints
ONE JSON line.
"""
import argparse
import hashlib
import json
import os
import shutil
import socket
import statistics
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "parallel-computation-of-an-inverted-index-using-map-reduce_amd")
sys.path.insert(0, os.path.join(PKG, "bindings"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
K1_TEXT_RAW_PER_BYTE = 0.595  # raw FETCH_SIZE bytes per text byte of K1b's streamed reads (r3 calibration)
LETTERS = "abcdefghijklmnopqrstuvwxyz"

WORKLOADS = {
    "config3": dict(bytes=10_000_000_000, files=10_000, vocab=1_000_000, seed=3,
                    label="zipf 10 GB x 10^4 files, vocab 10^6, seed 3"),
    "config5": dict(bytes=100_000_000_000, files=1_000_000, vocab=10_000_000, seed=5,
                    label="zipf 100 GB x 10^6 files, vocab 10^7, seed 5 (BASELINE configs[4])"),
    "config5share": dict(bytes=12_500_000_000, files=125_000, vocab=10_000_000, seed=5,
                         label="zipf 12.5 GB x 1.25*10^5 files, vocab 10^7, seed 5 (configs[4]-sized single-GPU corpus)"),
}


def log(msg):
    """Progress on stderr (a long CPU-baseline lane is not a hang)."""
    if os.environ.get("RANK", "0") == "0":
        print("bench: %s" % msg, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="config3")
    p.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                   help="N > 1: shard one corpus over the ranks (strong) or one corpus per rank (weak)")
    p.add_argument("--bytes", type=float, default=None, help="override the workload's corpus bytes")
    p.add_argument("--files", type=int, default=None)
    p.add_argument("--vocab", type=int, default=None)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--cpu-baseline", choices=["quick", "none"], default="quick")
    p.add_argument("--cpu-slice-kb", type=int, default=25,
                   help="file size of the reference's quick 360-file slice (median of 5 per lane)")
    p.add_argument("--cpu-protocol-kb", type=int, default=1000,
                   help="file size of BASELINE.md's protocol slice (360 files x 1 MB), one run of the reference at "
                        "M = cores / R = 26: cpu_baseline.value (0 = skip; minutes per run)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--gen-threads", type=int, default=16)
    p.add_argument("--io-bytes", type=float, default=2e9,
                   help="bytes of the corpus written to files for the file-reader and end-to-end legs (0 = skip)")
    p.add_argument("--letter-split", choices=["balanced", "reference"], default="reference",
                   help="letter ownership of the N>1 exchange: the reference's 26/N reducer split (main.c:129-130, "
                        "default) or histogram-balanced ranges (SURVEY §8 f4)")
    p.add_argument("--rank-share", default=None, metavar="r/N",
                   help="one GPU: index rank r's ii_partition share of the workload strong-scaled over N GPUs, "
                        "with its global file ids")
    a = p.parse_args()
    a.share = None
    if a.rank_share:
        r, _, n = a.rank_share.partition("/")
        a.share = (int(r), int(n))
        if not (a.share[1] >= 1 and 0 <= a.share[0] < a.share[1]):
            p.error("--rank-share r/N needs 0 <= r < N")
    if a.no_cpu_baseline:
        a.cpu_baseline = "none"
    w = WORKLOADS[a.workload]
    a.custom = any(v is not None for v in (a.bytes, a.files, a.vocab, a.seed))
    a.bytes = int(a.bytes if a.bytes is not None else w["bytes"])
    a.files = a.files if a.files is not None else w["files"]
    a.vocab = a.vocab if a.vocab is not None else w["vocab"]
    a.seed = a.seed if a.seed is not None else w["seed"]
    return a


def launch_ranks(a):
    """N > 1 outside torch.distributed: one child launcher, N ranks, its rc."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def host_cores():
    """CPU threads this job may use: the box exports OMP_NUM_THREADS as its
    per-GPU CPU share (os.cpu_count() is the whole machine there)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return max(1, n)


def libii_sha16():
    h = hashlib.sha256()
    with open(os.path.join(PKG, "libii.so"), "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:16]


def pmc_traffic(build, shape):
    """HBM bytes per launch by kernel from the newest committed rocprofv3 PMC
    summary (profiles/*_pmc_traffic.json, made by profiles/pmc_traffic.py from
    this same bench command), only if it was measured on this very libii.so
    build and on this workload (shape = bytes, files, GPUs, rank share: a
    kernel's traffic per launch depends on its input); ({}, reason) otherwise."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")))
    if not files:
        return {}, "no PMC summary in profiles/"
    why = "no PMC summary of this libii.so build (%s) in profiles/" % build
    for f in reversed(files):  # the summary made on this very build, whichever file holds it
        try:
            d = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        line = d.get("bench_line", {})
        if line.get("libii_sha16") != build:
            continue
        cfg = line.get("config", {})
        if (cfg.get("bytes"), cfg.get("files"), line.get("n_gpus"), cfg.get("rank_share")) != shape:
            why = "%s was measured on another workload" % os.path.basename(f)
            continue
        return ({k: v for k, v in d["kernels"].items() if "traffic_bytes_per_launch" in v}, os.path.basename(f))
    return {}, why


# the kernels of the sort + segmented-reduce phase (K2 token sort + K3), by rocprof name prefix
# (prefixes: the template arguments that follow vary with the build, e.g. the key type)
PHASE_KERNELS = ("ii::k_sort0_compact", "ii::k_radix_scatter<false, 512, 16, true", "ii::k_msd_scatter", "ii::k_seg_hist",
                 "ii::k_onesweep", "ii::k_uniq_sweep", "ii::k_radix_scatter<false, 512, 16, false")


def kernel_entry(traffic, prefix):
    """The PMC summary's entry of the kernel whose name starts with prefix (template
    instances such as k_tok_emit<false, false> included), or {}."""
    for k, v in traffic.items():
        if k == prefix or k.startswith(prefix + "<"):
            return v
    return {}


def pmc_phase_bytes(traffic):
    """HBM bytes per step of the phase kernels from the PMC summary (per-launch
    traffic x launches per step; a step runs k_sort0_compact once)."""
    steps = kernel_entry(traffic, "ii::k_sort0_compact").get("dispatches_FETCH_SIZE")
    if not steps:
        return None
    tot = 0.0
    for k, v in traffic.items():
        if k.startswith(PHASE_KERNELS):
            tot += v["traffic_bytes_per_launch"] * v["dispatches_FETCH_SIZE"] / steps
    return tot


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


def write_files(text, off, nf, td):
    import numpy as np
    names = []
    for f in range(nf):
        p = os.path.join(td, "f%06d.txt" % f)
        np.asarray(text[int(off[f]):int(off[f + 1])]).tofile(p)
        names.append(p)
    with open(os.path.join(td, "list.txt"), "w") as fl:
        fl.write("%d\n%s\n" % (nf, "\n".join(names)))
    return names


def cpu_baseline(a, text, off, runs=5):
    """CPU baseline: the reference itself
    (oracle/_ref/tema1 = gcc -O2 main.c) on reference-feasible slices of the
    same generator — 360 files (its MAX_FILES, main.c:8):
      protocol_slice  BASELINE.md's slice, 360 x --cpu-protocol-kb (1000) KB, at
                      M = cores / R = 26, one run (its O(T*V) reducer takes
                      minutes on a 10^6 vocabulary): `value` when it ran
      reference_lanes 360 x --cpu-slice-kb (25) KB at M = cores / R = 26,
                      M = R = cores and (SURVEY §8d's M = nproc) M = the CPUs of
                      this process's affinity set / R = 26, median of `runs`
                      each, and the as-shipped ASan build (Makefile:2) once for
                      context
    and the multithreaded hash-based restatement (oracle ii_oracle_index_mt,
    bit-exact) over the WHOLE corpus with `cores` threads."""
    import ii_ctypes
    cores = host_cores()
    ref = os.path.join(REPO, "oracle", "_ref", "tema1")
    asan = os.path.join(REPO, "oracle", "_ref", "tema1_asan")
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    # BASELINE.md asks for M = nproc: nproc here counts the whole machine's CPUs (256 on the GPU box),
    # of which one single-GPU job is granted a share — the box exports it as OMP_NUM_THREADS (16).
    # M and the restatement's threads use that share; the reference's map phase does not scale with M
    # anyway (shared-FILE locks) and its R is capped by the 26 letters.
    out = {"unit": "GB/s", "cores": cores, "nproc": os.cpu_count(), "affinity_cpus": affinity,
           "cores_basis": "threads granted to this job (OMP_NUM_THREADS, the box's per-GPU CPU share); "
                          "nproc counts the whole machine"}
    sl_files, sl_bytes = 360, 360 * 1000 * a.cpu_slice_kb
    st, so = ii_ctypes.zipf_corpus(sl_bytes, sl_files, a.vocab, a.seed + 77, threads=min(8, cores))
    m_ok = safe_mappers([int(so[f + 1] - so[f]) for f in range(sl_files)], cores)
    lanes = []
    if os.path.exists(ref):
        td = tempfile.mkdtemp(prefix="ii_cpu_")
        try:
            write_files(st, so, sl_files, td)

            def timed(binary, M, R, wd=td):
                t0 = time.perf_counter()
                pr = subprocess.Popen([binary, str(M), str(R), "list.txt"], cwd=wd, stdout=subprocess.DEVNULL,
                                      stderr=subprocess.DEVNULL)
                while True:  # a progress line every 30 s (a long slice is not a hang)
                    try:
                        rc = pr.wait(timeout=30)
                        break
                    except subprocess.TimeoutExpired:
                        log("cpu baseline: %s still running (%.0f s)" % (os.path.basename(binary), time.perf_counter() - t0))
                        if time.perf_counter() - t0 > 1800:
                            pr.kill()
                            raise
                if rc != 0:
                    raise subprocess.CalledProcessError(rc, binary)
                return time.perf_counter() - t0

            # SURVEY §8d's M = nproc lane too: every CPU this process may run on (the affinity set), R = 26
            m_aff = safe_mappers([int(so[f + 1] - so[f]) for f in range(sl_files)], affinity) \
                if affinity and affinity > cores else None
            for M, R in [(m_ok, 26), (m_ok, m_ok)] + ([(m_aff, 26)] if m_aff else []):
                log("cpu baseline: reference M=%d R=%d x%d" % (M, R, runs))
                ts = [timed(ref, M, R) for _ in range(runs)]
                lanes.append({"binary": "tema1 (gcc -O2 main.c)", "M": M, "R": R, "runs": runs,
                              "median_s": round(statistics.median(ts), 3), "all_s": [round(x, 3) for x in ts],
                              "GBps": round(sl_bytes / statistics.median(ts) / 1e9, 6)})
            if os.path.exists(asan):
                log("cpu baseline: reference as shipped (ASan)")
                t = timed(asan, m_ok, 26)
                lanes.append({"binary": "tema1_asan (as shipped, -fsanitize=address -g)", "M": m_ok, "R": 26,
                              "runs": 1, "median_s": round(t, 3), "GBps": round(sl_bytes / t / 1e9, 6)})
        finally:
            shutil.rmtree(td, ignore_errors=True)
        best = max([x for x in lanes if x["binary"].startswith("tema1 (")], key=lambda x: x["GBps"])
        out.update({"value": best["GBps"], "kind": "reference", "M": best["M"], "R": best["R"],
                    "sample": "reference binary on 360 files x %d KB (%.1f MB) of the same generator (vocab %d); "
                              "median of %d" % (a.cpu_slice_kb, sl_bytes / 1e6, a.vocab, runs), "reference_lanes": lanes})
        if a.cpu_protocol_kb > 0:
            pb = 360 * 1000 * a.cpu_protocol_kb
            pt, po = ii_ctypes.zipf_corpus(pb, 360, a.vocab, a.seed + 77, threads=min(8, cores))
            pm = safe_mappers([int(po[f + 1] - po[f]) for f in range(360)], cores)
            td = tempfile.mkdtemp(prefix="ii_cpu_")
            try:
                write_files(pt, po, 360, td)
                del pt
                log("cpu baseline: reference on the protocol slice (360 x %d KB) M=%d R=26, one run"
                    % (a.cpu_protocol_kb, pm))
                t = timed(ref, pm, 26, td)
            finally:
                shutil.rmtree(td, ignore_errors=True)
            ps = {"binary": "tema1 (gcc -O2 main.c)", "M": pm, "R": 26, "runs": 1, "seconds": round(t, 2),
                  "bytes": pb, "GBps": round(pb / t / 1e9, 6)}
            out["protocol_slice"] = ps
            out.update({"value": ps["GBps"], "M": pm, "R": 26,
                        "sample": "reference binary on BASELINE.md's protocol slice: 360 files x %d KB (%.0f MB) of the "
                                  "same generator (vocab %d), M = %d / R = 26, one run (%.1f s)"
                                  % (a.cpu_protocol_kb, pb / 1e6, a.vocab, pm, t)})
    # the bit-exact multithreaded restatement at full size
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_py import oracle_index
    n = len(off) - 1
    log("cpu baseline: multithreaded restatement over %.3g GB, %d threads" % (int(off[-1]) / 1e9, cores))
    t0 = time.perf_counter()
    oracle_index(text, off, list(range(n)), threads=cores)
    dt = time.perf_counter() - t0
    full = {"kind": "port", "what": "oracle ii_oracle_index_mt (hash-based restatement, bit-exact), whole corpus",
            "threads": cores, "bytes": int(off[-1]), "seconds": round(dt, 2), "GBps": round(int(off[-1]) / dt / 1e9, 4)}
    out["restatement_full"] = full
    if "value" not in out:  # no reference binary on this host: the restatement is the baseline
        out.update({"value": full["GBps"], "kind": "port", "sample": full["what"]})
    return out


def config2_lane(idx, runs=5):
    """BASELINE configs[1] as-is: the reference's own fixture (test.txt, 355
    chapter files of 6 novels, 5.76 MB; committed as tests/golden/config2.tar.xz
    with the reference binary's output), the reference binary (oracle/_ref/tema1)
    at M = min(cores, 8) / R = 26 — SURVEY's best lane — median of `runs`,
    beside this GPU's device-resident map + reduce of the same files (median of
    `runs`), whose output is checked byte for byte against the fixture."""
    import tarfile
    import numpy as np
    import torch
    cores = host_cores()
    ref = os.path.join(REPO, "oracle", "_ref", "tema1")
    td = tempfile.mkdtemp(prefix="ii_c2_")
    try:
        with tarfile.open(os.path.join(REPO, "tests", "golden", "config2.tar.xz"), "r:xz") as tar:
            tar.extractall(td)
        names = open(os.path.join(td, "list.txt")).read().split()
        paths = [os.path.join(td, x) for x in names[1:1 + int(names[0])]]
        expected = {l: open(os.path.join(td, "expected", l + ".txt"), "rb").read() for l in LETTERS}
        out = {"fixture": "test.txt (355 files, reference fixture)", "cores": cores}
        sizes = [os.path.getsize(x) for x in paths]
        B = sum(sizes)
        out["bytes"] = B
        if os.path.exists(ref):
            M = safe_mappers(sizes, min(cores, 8))
            ts = []
            for _ in range(runs):  # (the list's paths are relative to td; outputs land in td)
                t0 = time.perf_counter()
                subprocess.run([ref, str(M), "26", "list.txt"], cwd=td, check=True, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL)
                ts.append(time.perf_counter() - t0)
            out["reference"] = {"binary": "tema1 (gcc -O2 main.c)", "M": M, "R": 26, "runs": runs,
                                "median_s": round(statistics.median(ts), 4), "all_s": [round(x, 4) for x in ts],
                                "GBps": round(B / statistics.median(ts) / 1e9, 6)}
        # the GPU on the same files: text resident in HBM (files back to back, '\n' after each)
        data = [open(x, "rb").read() for x in paths]
        buf = bytearray()
        starts = []
        for d in data:
            starts.append(len(buf))
            buf += d + b"\n"
        n = len(buf)
        d_text = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        d_text[:n].copy_(torch.frombuffer(buf, dtype=torch.uint8))  # (a bytearray: writable, no copy)
        fs = np.asarray(starts, dtype=np.uint64)
        ids = np.arange(len(paths), dtype=np.uint32)
        ts = []
        for it in range(runs + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            idx.map_device(d_text.data_ptr(), n, fs, ids)
            idx.reduce(copy_text=False)
            torch.cuda.synchronize()
            if it:
                ts.append(time.perf_counter() - t0)
        idx.map_device(d_text.data_ptr(), n, fs, ids)
        idx.reduce(copy_text=True)
        ok = all(idx.letter_text(i) == expected[l] for i, l in enumerate(LETTERS))
        out["gpu"] = {"what": "map + reduce, device-resident text, one MI355X", "runs": runs,
                      "median_ms": round(statistics.median(ts) * 1e3, 3), "GBps": round(B / statistics.median(ts) / 1e9, 4),
                      "bit_exact_vs_reference": ok}
        return out
    finally:
        shutil.rmtree(td, ignore_errors=True)


def io_legs(idx, text, off, io_bytes, cores):
    """Beside `value`, never as it: the first files of the corpus (<= io_bytes)
    are written to a scratch directory (page cache warm: just written), then
      io  — ii_map_files reads them (pipelined pread into pinned windows +
            async H2D, 16 readers) and maps them; best of 2;
      e2e — the drop-in CLI `ii_index M R list.txt` in a fresh process: list
            file -> stat -> read + upload -> index -> a.txt..z.txt written to
            disk, process start and HIP initialisation included."""
    nf = 0
    while nf < len(off) - 1 and off[nf + 1] <= io_bytes:
        nf += 1
    if nf == 0:
        return None, None
    td = tempfile.mkdtemp(prefix="ii_io_")
    try:
        paths = write_files(text, off, nf, td)
        best = None
        for _ in range(2):
            t0 = time.perf_counter()
            idx.map_files(paths, nthreads=16)
            wall = time.perf_counter() - t0
            st = idx.stats()
            if best is None or wall < best[0]:
                best = (wall, st.io_ms, st.io_bytes, st.ms_map)
        wall, io_ms, io_b, map_ms = best
        io = {"files": nf, "bytes": int(off[nf]), "threads": 16, "read_upload_ms": round(io_ms, 2),
              "read_upload_GBps": round(io_b / (io_ms * 1e-3) / 1e9, 2) if io_ms > 0 else None,
              "map_files_ms": round(wall * 1e3, 2), "map_files_GBps": round(int(off[nf]) / wall / 1e9, 2),
              "k1_ms": round(map_ms, 2), "page_cache": "warm"}
        M = min(16, cores)
        runs = []
        for _ in range(2):
            wd = tempfile.mkdtemp(prefix="ii_e2e_", dir=td)
            t0 = time.perf_counter()
            r = subprocess.run([os.path.join(PKG, "ii_index"), str(M), "26", os.path.join(td, "list.txt")], cwd=wd,
                               stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=300)
            runs.append(time.perf_counter() - t0)
            if r.returncode != 0:
                return io, {"error": r.stderr.decode()[-300:]}
            out_b = sum(os.path.getsize(os.path.join(wd, l + ".txt")) for l in LETTERS)
        e2e = {"what": "ii_index %d 26 list.txt (fresh process: HIP init, stat, read, index, write a..z.txt)" % M,
               "files": nf, "bytes": int(off[nf]), "out_bytes": out_b, "wall_s": [round(x, 3) for x in runs],
               "GBps": round(int(off[nf]) / min(runs) / 1e9, 3), "page_cache": "warm"}
        return io, e2e
    finally:
        shutil.rmtree(td, ignore_errors=True)


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    import numpy as np
    import torch
    import torch.distributed as dist
    import ii_ctypes
    import ii_dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus == 1 and world > 1:
        a.gpus = world
    if a.gpus != world:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (a.gpus, world))
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
    strong = a.scaling == "strong" or world == 1
    if a.share and world > 1:
        sys.exit("bench.py: --rank-share runs one rank's share on one GPU (--gpus 1)")
    if a.workload == "config5" and world == 1 and not a.share and not a.custom:
        sys.exit("bench.py: config5 (100 GB) is the 8-GPU workload: --gpus 8, or --rank-share r/8 on one GPU")

    # ---- this rank's files, generated on the host, then to HBM
    log("generating %s (%d rank(s), %s scaling%s)" % (a.workload, world, "strong" if strong else "weak",
                                                    ", share %d/%d" % a.share if a.share else ""))
    t0 = time.perf_counter()
    if a.share:  # one rank's ii_partition share (main.c:300-323), global ids
        layout = ii_ctypes.zipf_layout(a.bytes, a.files, a.seed)
        sizes = [int(x) for x in (layout[1:] - layout[:-1])]
        order, sb, se = ii_ctypes.partition(sizes, a.share[1])
        ids = sorted(order[sb[a.share[0]]:se[a.share[0]]])
        text, off = ii_ctypes.zipf_shard(a.bytes, a.files, a.vocab, a.seed, ids, threads=a.gen_threads)
        id_bound = a.files
        total_bytes = int(off[-1])
    elif strong:
        layout = ii_ctypes.zipf_layout(a.bytes, a.files, a.seed)
        if world > 1:  # the reference's size heuristic, one shard per GPU (main.c:300-323)
            sizes = [int(x) for x in (layout[1:] - layout[:-1])]
            order, sb, se = ii_ctypes.partition(sizes, world)
            ids = sorted(order[sb[rank]:se[rank]])
            text, off = ii_ctypes.zipf_shard(a.bytes, a.files, a.vocab, a.seed, ids, threads=a.gen_threads)
        else:
            ids = list(range(a.files))
            text, off = ii_ctypes.zipf_corpus(a.bytes, a.files, a.vocab, a.seed, threads=a.gen_threads)
        id_bound = a.files
        total_bytes = a.bytes
    else:
        text, off = ii_ctypes.zipf_corpus(a.bytes, a.files, a.vocab, a.seed + 1000 * rank, threads=a.gen_threads)
        ids = list(range(rank * a.files, (rank + 1) * a.files))  # rank r owns files [r*F, (r+1)*F)
        id_bound = world * a.files
        total_bytes = a.bytes * world
    gen_s = time.perf_counter() - t0
    nbytes = int(off[-1])
    d_text = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
    if nbytes:
        d_text[:nbytes].copy_(torch.from_numpy(text[:nbytes]))
    torch.cuda.synchronize()
    # the file table as contiguous arrays: passed to ii_map_device in place every step
    file_start = np.ascontiguousarray(off[:-1], dtype=np.uint64)
    file_ids = np.ascontiguousarray(ids, dtype=np.uint32)

    idx = ii_ctypes.Index(local if world > 1 else 0)
    owned = [(0, 26)]
    local_st = [None]  # N > 1: the rank's stats after its map + local reduce (the owner's import maps again)

    def keep_local(ix):
        local_st[0] = ix.stats()

    def step(copy_text=False, capture=False):
        idx.map_device(d_text.data_ptr(), nbytes, file_start, file_ids)
        if world > 1:  # local reduce -> letter-range all-to-allv (RCCL) -> owner merge + format
            _, (lo, hi) = ii_dist.exchange_and_reduce(idx, id_bound, balanced=a.letter_split == "balanced",
                                                      copy_text=copy_text, on_local=keep_local if capture else None)
            owned[0] = (lo[rank], hi[rank])
        else:
            idx.reduce(copy_text=copy_text)

    log("warmup %d + timed %d steps" % (a.warmup, a.steps))
    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scatter_ms, emit_ms, phase_ms = [], [], []
    for i in range(a.steps):
        step(capture=world > 1 and i == a.steps - 1)
        if world == 1:
            st = idx.stats()
            scatter_ms.append(st.scatter_ms_avg)
            emit_ms.append(st.emit_ms)
            phase_ms.append(st.ms_sort + st.ms_reduce)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    # the kernel figures (roofline, phases, counts) of an N > 1 line describe this rank's map + local
    # reduce of the last timed step; after the exchange the context holds the owner's import instead
    st = idx.stats() if world == 1 else local_st[0]
    if world > 1:
        scatter_ms, emit_ms, phase_ms = [st.scatter_ms_avg], [st.emit_ms], [st.ms_sort + st.ms_reduce]
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / a.steps * 1e3
    value = total_bytes * a.steps / dt / 1e9

    # ---- --rank-share: what the rank does before the exchange (map + local reduce + export), timed apart
    export_leg = None
    if a.share:
        parts = a.share[1]
        send = None
        ts = []
        for it in range(a.warmup + a.steps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            idx.map_device(d_text.data_ptr(), nbytes, file_start, file_ids)
            idx.reduce_local()
            sizes = idx.export_plan(parts)
            soff, stot = ii_dist.prefix(sizes)
            if send is None or send.numel() < stot:
                send = torch.empty(max(stot, 8), dtype=torch.uint8, device="cuda")
            idx.export(parts, send.data_ptr(), soff)
            torch.cuda.synchronize()
            if it >= a.warmup:
                ts.append(time.perf_counter() - t1)
        export_leg = {"what": "map + ii_reduce_local + ii_export_plan + ii_export (%d parts, the reference's "
                              "reducer letters)" % parts, "ms": round(statistics.median(ts) * 1e3, 3),
                      "GBps": round(total_bytes / statistics.median(ts) / 1e9, 3), "send_bytes": int(sum(sizes))}

    # ---- outside the timed region: the index itself, against the oracle's hashes
    verified, verify_note, letter_sha = None, None, {}
    if not a.no_verify:
        log("verifying the index against the oracle's hashes")
        step(copy_text=True)
        lo, hi = owned[0]
        mine = {LETTERS[l]: hashlib.sha256(idx.letter_text(l)).hexdigest() for l in range(lo, hi)}
        if world > 1:
            allh = [None] * world
            dist.all_gather_object(allh, mine)
            for h in allh:
                letter_sha.update(h)
        else:
            letter_sha = mine
        if rank == 0:
            db = json.load(open(os.path.join(REPO, "tests", "golden", "bench_hashes.json")))["workloads"]
            key = a.workload + ("/share%dof%d" % a.share if a.share else "")
            exp = db.get(key)
            if a.custom or not strong or exp is None:
                verify_note = "no oracle hashes for this corpus (custom size or weak scaling)"
            else:
                bad = [l for l in LETTERS if letter_sha.get(l) != exp["letters"][l]["sha256"]]
                verified = not bad and len(letter_sha) == 26
                verify_note = "26 letters match the oracle (tests/golden/bench_hashes.json %s)" % key if verified else \
                    "letters differ from the oracle: %s" % "".join(bad)

    if rank == 0:
        build = libii_sha16()
        sc_ms = sum(scatter_ms) / len(scatter_ms)
        sc_achieved = st.scatter_bytes / (sc_ms * 1e-3) / 1e9 if sc_ms > 0 else 0.0
        em_ms = sum(emit_ms) / len(emit_ms)
        em_achieved = st.emit_bytes / (em_ms * 1e-3) / 1e9 if em_ms > 0 else 0.0
        traffic, traffic_src = pmc_traffic(build, (a.bytes if strong else a.bytes * world, a.files, world,
                                                   "%d/%d" % a.share if a.share else None))
        # sort + segmented-reduce phase (K2 token sort + K3 unique), three byte counts:
        #  impl:   the bytes this build's kernels must move —
        #          the first pass reads T records (4 B from narrow chunks' u32 word slots,
        #          8 B from the others) and writes the T_k kept ones (st.sort0_bytes), the passes after it as the
        #          library counts them (st.sort_bytes: the packed form's u32 bucket
        #          passes), K3 reads the sorted records once (u32 in the packed form)
        #          and writes the pairs, the posting offsets P (every word start and
        #          every 64th pair) and the per-word start / end arrays
        #  survey: SURVEY §8d's model with 8-B records — first pass 8T + 8T_k, 16 T_k
        #          per later pass, the unique pass 8 T_k + 8 U + 16 V — which charges
        #          the packed passes for u64 records they do not move (secondary)
        #  pmc:    HBM bytes the counters saw for the phase's kernels (rocprofv3
        #          FETCH_SIZE x correction + WRITE_SIZE, profiles/*_pmc_traffic.json
        #          of this very build), when there is such a summary: then `frac` is
        #          pmc_frac (SURVEY §8d defines achieved HBM by the counters), else impl
        T, Tk, U, V = st.tokens, st.sorted_records, st.pairs, st.words
        sp = max(1, st.sort_passes)
        survey_b = 8 * T + 8 * Tk + sp * 16 * Tk + 8 * Tk + 8 * U + 16 * V
        k3_read = (4 if st.sort_packed else 8) * Tk  # the packed form's K3 reads u32 records
        # (the pairs: 4 B each when K3 wrote the compact form, plus the word key of every 64th)
        pair_b = (4 * U + 4 * (U // 64)) if st.pair_bytes == 4 else 8 * U
        impl_b = st.sort0_bytes + st.sort_bytes + k3_read + pair_b + 8 * (V + U // 64) + 16 * V
        ph_ms = sum(phase_ms) / len(phase_ms)
        ph_gbs = impl_b / (ph_ms * 1e-3) / 1e9 if ph_ms > 0 else 0.0
        pmc_b = pmc_phase_bytes(traffic) if traffic else None
        impl_frac = ph_gbs / HBM_PEAK_GBS
        pmc_frac = pmc_b / (ph_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if pmc_b and ph_ms > 0 else None
        # K1b: SURVEY §8d's tokenize model (B + 12 T, 12-B canonical records) beside the library's
        # B + 8 T; PMC traffic split into the streamed text and the hot-table probe lines: the text is
        # read with 16-B loads whose 128-B requests FETCH_SIZE tallies at 64 B (x2, MI355X_MICROARCH.md),
        # the probes' 64-B requests are tallied at full size (no x2).  The text share of the raw
        # FETCH_SIZE is calibrated on the probe-free K1b variant (tools/k1_ablate, round 3:
        # TCC_EA0_RDREQ 9.3e6 128-B requests = 0.595 raw FETCH bytes per text byte, incl. halos and
        # the K1c tail's re-reads; profiles/r3_k1_pmc_1GB.txt)
        B_emit = st.bytes
        k1_survey_b = B_emit + 12 * T
        k1 = kernel_entry(traffic, "ii::k_tok_emit")
        k1_split = None
        if "read_raw_bytes_per_launch" in k1:
            raw = k1["read_raw_bytes_per_launch"]
            text_raw = min(raw, K1_TEXT_RAW_PER_BYTE * B_emit)
            probe = raw - text_raw
            wr = k1["write_bytes_per_launch"]
            k1_split = {"traffic_model": round(2 * text_raw + probe + wr), "traffic_model_text": round(2 * text_raw),
                        "traffic_model_probe": round(probe), "traffic_model_write": round(wr),
                        "probe_bytes_per_text_byte": round(probe / B_emit, 3) if B_emit else None}
        cpu = None
        if a.cpu_baseline != "none" and world == 1:
            cpu = cpu_baseline(a, text, off)
            log("configs[1] lane: the reference and the GPU on test.txt")
            cpu["config2"] = config2_lane(idx)
        log("file reader and end-to-end legs")
        io, e2e = io_legs(idx, text, off, a.io_bytes, host_cores()) if world == 1 and a.io_bytes > 0 else (None, None)
        wl = WORKLOADS[a.workload]
        workload = "%s: %s" % (a.workload, wl["label"] if not a.custom else "zipf %.4g GB x %d files, vocab %d, seed %d"
                               % (a.bytes / 1e9, a.files, a.vocab, a.seed))
        if a.share:
            workload += "; rank %d's share of %d (ii_partition, global ids)" % a.share
        elif a.workload == "config3":
            workload += " (BASELINE configs[3]: sharded over %d GPUs by ii_partition)" % world if world > 1 and strong \
                else " (BASELINE configs[2])" if world == 1 else " per rank (weak scaling)"
        elif a.workload == "config5" and world > 1 and strong:
            workload += ", sharded over %d GPUs by ii_partition" % world
        line = {
            "metric": "indexed input GB/s (whole node) + % of HBM peak BW",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            # strong: one corpus whatever N (total work fixed); weak: a corpus per rank
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic Zipf corpus (tools/iigen.c, s~1), device-resident",
            "verified": verified,
            "verify": verify_note,
            "config": {"workload": workload, "bytes": a.bytes if strong else a.bytes * world,
                       "files": a.files if strong else a.files * world, "vocab": a.vocab, "seed": a.seed,
                       "bytes_rank0": nbytes, "files_rank0": len(ids),
                       "rank_share": "%d/%d" % a.share if a.share else None,
                       "parallelism": "files by size over %d GPU(s) + letter-range all-to-allv" % world
                       if world > 1 else "one GPU",
                       "letter_split": a.letter_split if world > 1 or a.share else None},
            # dominant kernel: the tokenizer (K1b); algorithmic bytes per launch = SURVEY §8d's
            # B + 12*T (12-B canonical records; `frac`), and the library's B + 8*T beside it
            "roofline": {"bound": "hbm", "kernel": "k_tok_emit (K1b tokenizer)",
                         "achieved": round(k1_survey_b / (em_ms * 1e-3) / 1e9, 1) if em_ms > 0 else 0.0,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(k1_survey_b / (em_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if em_ms > 0 else 0.0,
                         "bytes_per_launch": k1_survey_b, "model": "SURVEY §8d: B + 12 T",
                         "achieved_b8t": round(em_achieved, 1), "frac_b8t": round(em_achieved / HBM_PEAK_GBS, 4),
                         "bytes_per_launch_b8t": st.emit_bytes,
                         # measured: PMC FETCH_SIZE x2 + WRITE_SIZE per launch (MI355X_MICROARCH.md's gfx950
                         # correction) of this very build, or null
                         "traffic": round(k1["traffic_bytes_per_launch"]) if "traffic_bytes_per_launch" in k1
                         else None,
                         # a MODEL split of the measured counters (not measured itself): x2 on the streamed text
                         # only, its share of raw FETCH_SIZE calibrated on the round-3 probe-free variant
                         # (K1_TEXT_RAW_PER_BYTE, profiles/r3_k1_pmc_1GB.txt), the probes' 64-B requests unscaled
                         "traffic_model": k1_split["traffic_model"] if k1_split else None,
                         "traffic_model_text": k1_split["traffic_model_text"] if k1_split else None,
                         "traffic_model_probe": k1_split["traffic_model_probe"] if k1_split else None,
                         "traffic_model_write": k1_split["traffic_model_write"] if k1_split else None,
                         "traffic_model_calibration": "round-3 K1b, profiles/r3_k1_pmc_1GB.txt",
                         "probe_bytes_per_text_byte": k1_split["probe_bytes_per_text_byte"] if k1_split else None,
                         "traffic_raw": round(k1["traffic_raw_bytes_per_launch"]) if "traffic_raw_bytes_per_launch" in k1
                         else None,
                         "traffic_note": "FETCH_SIZE counts Infinity-Cache hits too (MI355X_MICROARCH.md): the 8 MB "
                                         "hot table's probe lines are mostly served on-die, not by HBM",
                         "traffic_source": traffic_src, "ms_per_launch": round(em_ms, 4)},
            "roofline_sort": {"bound": "hbm", "kernel": "k_radix_scatter (token sort passes)",
                              "achieved": round(sc_achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(sc_achieved / HBM_PEAK_GBS, 4),
                              "bytes_per_launch": st.scatter_bytes, "ms_per_launch": round(sc_ms, 4)},
            "roofline_sort_phase": {"bound": "hbm", "phase": "token sort + segmented unique (K2 + K3)",
                                    "model": "PMC counters (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of this build)"
                                    if pmc_frac is not None else "bytes this build's kernels must move (impl)",
                                    "achieved": round((pmc_frac if pmc_frac is not None else impl_frac) * HBM_PEAK_GBS, 1),
                                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": round(pmc_frac if pmc_frac is not None else impl_frac, 4),
                                    "impl_frac": round(impl_frac, 4), "impl_achieved": round(ph_gbs, 1),
                                    "bytes_per_step": impl_b, "survey_bytes_per_step": survey_b,
                                    "survey_frac": round(survey_b / (ph_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                    if ph_ms > 0 else 0.0,
                                    "pmc_bytes_per_step": round(pmc_b) if pmc_b else None,
                                    "pmc_frac": round(pmc_frac, 4) if pmc_frac is not None else None,
                                    "ms_per_step": round(ph_ms, 4),
                                    "first_pass": {"kernel": "k_sort0_compact", "ms": round(st.sort0_ms, 4),
                                                   "bytes": st.sort0_bytes,
                                                   "achieved": round(st.sort0_bytes / (st.sort0_ms * 1e-3) / 1e9, 1)
                                                   if st.sort0_ms > 0 else 0.0}},
            "cpu_baseline": cpu,
            "io": io,
            "e2e": e2e,
            "kernel_figures_of": "this run" if world == 1 else
            "rank 0's map + local reduce (last timed step; the owner's import maps again)",
            "phases_ms": {k: round(getattr(st, k), 3) for k in
                          ["ms_map", "ms_dict", "ms_sort", "ms_reduce", "ms_order", "ms_format", "ms_total",
                           "emit_ms", "resolve_ms"]},
            "counts": {"tokens": st.tokens, "pairs": st.pairs, "words": st.words, "long_tokens": st.long_tokens,
                       "out_bytes": st.out_bytes, "sort_passes": st.sort_passes, "table_cap": st.table_cap,
                       "resolved_tokens": st.resolved_tokens, "sorted_records": st.sorted_records,
                       "sort_packed": st.sort_packed, "sort_key_bits": st.sort_key_bits,
                       "sort_id_bits": st.sort_id_bits, "files": len(ids)},
            "export": export_leg,
            "output_letter_sha256": letter_sha if letter_sha else None,
            "libii_sha16": build,
            "gen_seconds": round(gen_s, 2),
        }
        print(json.dumps(line), flush=True)
    idx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
