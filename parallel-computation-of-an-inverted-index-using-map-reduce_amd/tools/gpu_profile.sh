#!/bin/bash
# gpu_profile.sh TAG — one GPU-box session for a milestone: the default bench
# line, rocprofv3 kernel statistics of the same bench, and the PMC HBM traffic
# passes (profiles/pmc_traffic.py).  Each step under its own time limit,
# chained with && (the first failure ends the session).  Results in
# gpurun_out/TAG/.
set -o pipefail
TAG=${1:-prof}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
echo "== bench" && \
timeout -k 10 500 python bench.py > "$OUT/bench.log" 2>&1 && tail -1 "$OUT/bench.log" | cut -c1-300 && \
echo "== rocprof" && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify > "$OUT/prof.log" 2>&1 && \
find "$OUT/prof" -name '*kernel_stats.csv' -exec head -8 {} \; | cut -c1-160 && \
echo "== pmc" && \
timeout -k 10 600 python3 profiles/pmc_traffic.py run "$OUT/pmc" --steps 3 --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify && \
python3 profiles/pmc_traffic.py summarize "$OUT/pmc" > "$OUT/pmc_traffic.json" && echo "pmc ok"
