#!/usr/bin/env python3
"""BASELINE.md's CPU protocol on the reference-feasible slice: 360 files x
FILE_KB KB of the bench generator (config3's vocabulary and seed + 77), the
reference binary (oracle/_ref/tema1 = gcc -O2 main.c) at M = cores / R = 26
and M = R = cores, median of RUNS each, and its as-shipped ASan build once.
Results are written as they come (JSON), so a long protocol is never lost.

    python3 tools/cpu_slice.py OUT.json [FILE_KB=1000] [RUNS=5]
"""
import json
import os
import platform
import shutil
import statistics
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "bindings"))
sys.path.insert(0, REPO)


def main():
    out_path = sys.argv[1]
    file_kb = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    runs = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    import bench
    import ii_ctypes
    cores = bench.host_cores()
    nf, nb = 360, 360 * 1000 * file_kb
    text, off = ii_ctypes.zipf_corpus(nb, nf, 1_000_000, 3 + 77, threads=min(8, cores))
    M = bench.safe_mappers([int(off[f + 1] - off[f]) for f in range(nf)], cores)
    res = {"what": "reference binary on 360 files x %d KB (%.1f MB) of the bench generator (vocab 10^6)" % (file_kb, nb / 1e6),
           "host": platform.node(), "cores": cores, "host_cpus": os.cpu_count(), "lanes": []}
    td = tempfile.mkdtemp(prefix="ii_slice_")
    try:
        bench.write_files(text, off, nf, td)
        lanes = [("tema1", M, 26, runs), ("tema1", M, M, runs), ("tema1_asan", M, 26, 1)]
        for binary, m, r, k in lanes:
            path = os.path.join(REPO, "oracle", "_ref", binary)
            ts = []
            for i in range(k):
                t0 = time.perf_counter()
                subprocess.run([path, str(m), str(r), "list.txt"], cwd=td, check=True, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL)
                ts.append(round(time.perf_counter() - t0, 3))
                print("%s M=%d R=%d run %d: %.2f s" % (binary, m, r, i + 1, ts[-1]), flush=True)
            med = statistics.median(ts)
            res["lanes"] = [x for x in res["lanes"] if (x["binary"], x["M"], x["R"]) != (binary, m, r)]
            res["lanes"].append({"binary": binary, "M": m, "R": r, "runs": k, "all_s": ts, "median_s": med,
                                 "MBps": round(nb / med / 1e6, 3)})
            json.dump(res, open(out_path, "w"), indent=1)
    finally:
        shutil.rmtree(td, ignore_errors=True)


if __name__ == "__main__":
    main()
