#!/usr/bin/env python3
"""Per-kernel averages of the counters that tools/gpu_pmc.sh collected (one
rocprofv3 --pmc pass per directory passN/) — the summaries committed as
profiles/*_sq_counters*.txt.

    python3 tools/sq_summary.py gpurun_out/TAG/sq

SQ_WAIT_ANY (parked on s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall)
and SQ_ACTIVE_INST_ANY (issuing) are disjoint and sum to SQ_WAVE_CYCLES
(MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import sys


def main(d):
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "/pass*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k in sorted(set(k for k, _ in agg)):
        print(k)
        for (kk, c), v in sorted(agg.items()):
            if kk == k:
                print("   %-28s %16.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main(sys.argv[1])
