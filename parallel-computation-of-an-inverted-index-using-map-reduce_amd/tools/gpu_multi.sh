#!/bin/bash
# gpu_multi.sh TAG — one GPU-box session for the N > 1 workloads: rank 0's and
# rank 7's share of configs[4] (--workload config5 --rank-share r/8: that
# rank's ii_partition files with their global ids, map + local reduce +
# export), then a 4-rank gloo rehearsal of the strong-scaling bench at
# configs[3] (four ranks share the card; the exchange goes through host
# memory, so its rate is not the node's).  Each step under its own time
# limit, chained with && (the first failure ends the session).
set -o pipefail
TAG=${1:-multi}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
echo "== config5 share 0/8" && \
timeout -k 10 400 python bench.py --workload config5 --rank-share 0/8 --steps 5 --warmup 2 --no-cpu-baseline \
    --io-bytes 0 > "$OUT/share0.log" 2>&1 && tail -1 "$OUT/share0.log" | cut -c1-200 && \
echo "== config5 share 7/8" && \
timeout -k 10 400 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 --no-cpu-baseline \
    --io-bytes 0 > "$OUT/share7.log" 2>&1 && tail -1 "$OUT/share7.log" | cut -c1-200 && \
echo "== gloo x4 config3" && \
II_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 4 --steps 3 --warmup 1 > "$OUT/gloo4.log" 2>&1 && \
tail -1 "$OUT/gloo4.log" | cut -c1-200
