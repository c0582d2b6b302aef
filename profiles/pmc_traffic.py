#!/usr/bin/env python3
"""HBM traffic per kernel launch from rocprofv3 PMC counters (MI355X_MICROARCH.md §HBM).

    python3 profiles/pmc_traffic.py run  OUT_DIR [bench args...]   # on the GPU box
    python3 profiles/pmc_traffic.py summarize OUT_DIR > profiles/<round>_pmc_traffic.json

`run` makes two separate counter passes over the same bench command (FETCH_SIZE
alone, then WRITE_SIZE alone: they cannot share a pass on gfx950), each under
`timeout -s KILL`.  `summarize` averages the counters per dispatch of every
kernel and applies the gfx950 correction: FETCH_SIZE counts half the bytes of
a wide (16 B/lane) streaming read, so the read side is calibrated on
k_tok_count when the run has it (its read bytes are known: the text, B bytes,
read once with 16-B loads; measured factor 1.93), else doubled as the guide
prescribes (II_PMC_FETCH_FACTOR overrides); WRITE_SIZE is taken as reported.
"""
import csv
import collections
import json
import os
import subprocess
import sys

KERNELS = "k_tok_emit|k_tok_count|k_tok_resolve|k_long_verify|k_sort0_compact|k_radix_scatter|k_msd_scatter|k_onesweep|k_seg_hist|k_radix_hist|k_uniq|k_fmt_posts"


def run(out, bench_args):
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    for ctr in ["FETCH_SIZE", "WRITE_SIZE"]:
        d = os.path.join(out, ctr.lower())
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--pmc", ctr, "--kernel-include-regex", KERNELS,
               "--output-format", "csv", "-d", d, "-o", "run", "--", "python3", "bench.py"] + bench_args
        with open(os.path.join(out, ctr.lower() + ".log"), "w") as log:
            r = subprocess.run(cmd, stdout=log, stderr=subprocess.STDOUT, env=env)
        if r.returncode != 0:
            sys.exit("pass %s failed (%d)" % (ctr, r.returncode))


def load(d):
    agg = collections.defaultdict(list)
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(root, f))):
                    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                    agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def summarize(out):
    agg = load(out)
    res = {}
    for (name, ctr), vals in agg.items():
        res.setdefault(name, {})[ctr] = sum(vals) / len(vals)
        res[name]["dispatches_" + ctr] = len(vals)
    # calibrate the read side on k_tok_count (known read bytes)
    meta = {}
    bench_log = os.path.join(out, "fetch_size.log")
    for line in open(bench_log):
        if line.startswith("{"):
            meta = json.loads(line)
    B = meta.get("config", {}).get("bytes_rank0")
    factor = float(os.environ.get("II_PMC_FETCH_FACTOR", "2.0"))
    if B and "ii::k_tok_count" in res and "FETCH_SIZE" in res["ii::k_tok_count"]:
        known = B
        factor = known / (res["ii::k_tok_count"]["FETCH_SIZE"] * 1024)
    for name, v in res.items():
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            rd = v["FETCH_SIZE"] * 1024 * factor
            v["read_bytes_per_launch"] = rd
            v["write_bytes_per_launch"] = v["WRITE_SIZE"] * 1024
            v["traffic_bytes_per_launch"] = rd + v["WRITE_SIZE"] * 1024
            # uncorrected: the correction is for wide coalesced streaming reads; a kernel whose
            # reads are partly random (K1b's table probes) lies between the two
            v["read_raw_bytes_per_launch"] = v["FETCH_SIZE"] * 1024
            v["traffic_raw_bytes_per_launch"] = v["FETCH_SIZE"] * 1024 + v["WRITE_SIZE"] * 1024
    print(json.dumps({"fetch_correction_factor": factor, "bench_line": meta, "kernels": res}, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3:])
    else:
        summarize(sys.argv[2])
