#!/bin/bash
# gpu_sel.sh TAG "PYTEST -k EXPR" [BENCH=1] — one GPU-box session while iterating:
# a selection of the -m gpu tests (pytest -k), then (optionally) the quick
# bench line and rocprofv3 kernel statistics.  Each GPU step under its own time
# limit, chained with && (the first failure ends the session).
set -o pipefail
TAG=${1:-sel}
SEL=${2:-}
BENCH=${3:-1}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
run_tests() {
    [ -n "$SEL" ] || return 0
    echo "== tests: $SEL"
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -k "$SEL" --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1
    local rc=$?
    tail -3 "$OUT/pytest_gpu.log"
    return $rc
}
run_bench() {
    [ "$BENCH" = "1" ] || return 0
    echo "== bench" && \
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --io-bytes 0 > "$OUT/bench.log" 2>&1 && \
    tail -1 "$OUT/bench.log" | cut -c1-300 && \
    echo "== rocprof" && \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify > "$OUT/prof.log" 2>&1 && \
    echo "rocprof ok"
}
run_tests && run_bench
