#!/bin/bash
# gpu_strong.sh TAG [BYTES] [G] — the per-rank share of strong scaling on one
# GPU: bench.py at BYTES (the 8-GPU share of configs[3] by default) under
# rocprofv3 kernel statistics, then the exchange phases of G logical shards
# (tools/exchange_timing.py).  Each GPU step under its own time limit.
set -o pipefail
TAG=${1:-strong}
BYTES=${2:-1.25e9}
G=${3:-8}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
FILES=$(python3 -c "print(max(1, int(float('$BYTES') / 1e6)))")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --bytes "$BYTES" --files "$FILES" --steps 10 --warmup 2 --no-cpu-baseline --io-bytes 0 \
    --no-verify > "$OUT/bench.log" 2>&1 && tail -1 "$OUT/bench.log" | cut -c1-200 && \
timeout -k 10 300 python3 parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools/exchange_timing.py \
    "$BYTES" "$G" 3 > "$OUT/exchange.log" 2>&1 && tail -3 "$OUT/exchange.log"
