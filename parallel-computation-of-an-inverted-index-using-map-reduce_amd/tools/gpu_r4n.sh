#!/bin/bash
# one session: the whole -m gpu suite, smoke(), then the N > 1 lines (configs[4] shares 0/8 and 7/8,
# the 4-rank gloo rehearsal of the strong-scaling bench)
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4n}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
bash $T/gpu_multi.sh $TAG
