#!/bin/bash
# gpu_quick.sh — one short GPU-box session while iterating: the -m gpu tests
# (optional), the bench line without the CPU baselines and io legs, and
# rocprofv3 kernel statistics of the same bench.  Each GPU step under its own
# time limit, chained with && (the first failure ends the session).
#   tools/gpu_quick.sh TAG [RUN_TESTS=1] [STEPS=10]
# Results land in gpurun_out/TAG/.
set -o pipefail
TAG=${1:-quick}
RUN_TESTS=${2:-1}
STEPS=${3:-10}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp

run_tests() {
    [ "$RUN_TESTS" = "1" ] || return 0
    echo "== tests"
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1
    local rc=$?
    tail -3 "$OUT/pytest_gpu.log"
    return $rc
}

run_tests && \
echo "== bench" && \
timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 2 --no-cpu-baseline --io-bytes 0 > "$OUT/bench.log" 2>&1 && \
tail -1 "$OUT/bench.log" | cut -c1-200 && \
echo "== rocprof" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps "$STEPS" --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify > "$OUT/prof.log" 2>&1 && \
echo "rocprof ok"
