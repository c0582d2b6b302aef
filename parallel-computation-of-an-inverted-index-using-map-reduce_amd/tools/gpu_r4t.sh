#!/bin/bash
# one session: k_onesweep_seg's look-back granules per lane (II_SEG_LBPER 1 / 2 / 4 builds) at config3
# and on the rank-7 share (its buckets hold ~190 tiles, config3's ~30)
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4t}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
r7() {  # r7 NAME ENV...
    local name=$1; shift
    echo "== rank 7 $name"
    env "$@" timeout -k 10 400 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 --no-cpu-baseline \
        --io-bytes 0 --no-verify > $OUT/r7_$name.log 2>&1 && tail -1 $OUT/r7_$name.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); p=d['phases_ms']; s=d['roofline_sort_phase']
print('value=%.1f ms/step=%.2f sort_phase=%.4f scat=%.3f ms_sort=%.3f ms_reduce=%.3f' % (
 d['value'], d['ms_per_step'], s['frac'], d['roofline_sort']['ms_per_launch'], p['ms_sort'], p['ms_reduce']))"
}
echo "== tests (lb4)" && \
II_LIB_VARIANT=lb4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "packed_sort or tiny_shapes or wide_top or lookback" > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
bash $T/gpu_env_ab.sh $TAG 10e9 10 - II_LIB_VARIANT=lb4 II_LIB_VARIANT=lb1 - II_LIB_VARIANT=lb4 && \
r7 base II_NONE=1 && r7 lb4 II_LIB_VARIANT=lb4 && r7 lb1 II_LIB_VARIANT=lb1
