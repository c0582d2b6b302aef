#!/bin/bash
# final validation of the round's build: the whole -m gpu suite, smoke(), the default bench line
# (with the PMC traffic of this libii.so), then the N > 1 lines (configs[4] shares, 4-rank gloo)
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4w}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
echo "== bench" && timeout -k 10 500 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-200 && \
bash $T/gpu_multi.sh $TAG
