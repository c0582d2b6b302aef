#!/bin/bash
# gpu_check.sh — one GPU-box session: parity tests, K1 ablation, bench line and
# rocprofv3 kernel statistics of the same bench command.  Every GPU step runs
# under its own time limit and the steps are chained with &&, so the first
# failure ends the session.
#   tools/gpu_check.sh TAG [STEPS] [SKIP_TESTS] [TEST_SELECTION]
# Results land in gpurun_out/TAG/.
set -o pipefail
TAG=${1:-run}
STEPS=${2:-10}
SKIP_TESTS=${3:-0}
SEL=${4:-tests}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
PKG="$ROOT/parallel-computation-of-an-inverted-index-using-map-reduce_amd"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp

run_tests() {
    [ "$SKIP_TESTS" = "1" ] && return 0
    echo "== tests"
    # shellcheck disable=SC2086
    timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1
    local rc=$?
    tail -3 "$OUT/pytest_gpu.log"
    return $rc
}
run_ablate() {
    [ -x "$PKG/k1_ablate" ] || return 0
    echo "== ablate"
    timeout -k 10 180 "$PKG/k1_ablate" 1000000000 1000 1000000 > "$OUT/k1_ablate.log" 2>&1
    local rc=$?
    cat "$OUT/k1_ablate.log"
    return $rc
}

run_tests && run_ablate && \
echo "== bench" && \
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 2 > "$OUT/bench.log" 2>&1 && \
tail -1 "$OUT/bench.log" && \
echo "== rocprof" && \
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps "$STEPS" --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify > "$OUT/prof.log" 2>&1 && \
tail -1 "$OUT/prof.log" && \
find "$OUT/prof" -name '*kernel_stats.csv' -exec head -16 {} \;
