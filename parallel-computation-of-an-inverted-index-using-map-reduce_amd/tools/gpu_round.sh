#!/bin/bash
# gpu_round.sh TAG "PYTEST -k EXPR" VARIANTS... — one GPU-box session of a
# milestone: a selection of the -m gpu tests, then same-box A/B bench lines of
# the working tree ("base") against libii_<variant>.so builds (tools/build_rev.sh)
# at configs[2] and at configs[4]'s last rank share, then rocprofv3 kernel
# statistics of the working tree.  Each GPU step under its own time limit,
# chained with && (the first failure ends the session).
set -o pipefail
TAG=${1:-round}
SEL=${2:-}
shift 2
VARS="base $*"
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
T="$ROOT/parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools"
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
run_tests && \
echo "== A/B config3" && bash "$T/gpu_ab.sh" "$TAG/ab3" 10000000000 10 $VARS && \
echo "== A/B config5 rank 7" && AB_ARGS="--workload config5 --rank-share 7/8" bash "$T/gpu_ab.sh" "$TAG/ab5r7" - 5 $VARS && \
echo "== rocprof" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify > "$OUT/prof.log" 2>&1 && \
echo "rocprof ok"
