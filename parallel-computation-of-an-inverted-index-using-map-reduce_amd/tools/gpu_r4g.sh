#!/bin/bash
# one session: the wide top digit and the paired first sort pass (II_S0_HALF=1) through the sort /
# parity tests, then A/B of the paired pass at the bench size, then the rank-7 share (now packed)
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "first_pass_forms or packed_sort or config5_shape or tiny_shapes or global_ids or large_vocab or bench_verify" \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
bash $T/gpu_env_ab.sh $TAG 10e9 10 - II_S0_HALF=1 - II_S0_HALF=1 && \
echo "== rank 7" && \
timeout -k 10 400 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 --no-cpu-baseline --io-bytes 0 > $OUT/r7_base.log 2>&1 && tail -1 $OUT/r7_base.log | cut -c1-400 && \
II_S0_HALF=1 timeout -k 10 400 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 --no-cpu-baseline --io-bytes 0 > $OUT/r7_half.log 2>&1 && tail -1 $OUT/r7_half.log | cut -c1-400
