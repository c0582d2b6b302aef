#!/bin/bash
# one session: k_seg_hist variants (II_SEGHIST 0 plain / 1 wave groups / 2 four copies) against the
# build of 3ef4667 (libii_r4j.so) at config3 and the rank-7 share, and the owner-merge timing of both
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4m}
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
print('value=%.1f ms/step=%.2f sort_phase=%.4f sort0=%.3f ms_sort=%.3f ms_reduce=%.3f emit=%.3f' % (
 d['value'], d['ms_per_step'], s['frac'], s['first_pass']['ms'], p['ms_sort'], p['ms_reduce'], p['emit_ms']))"
}
echo "== tests (II_SEGHIST=2)" && \
II_SEGHIST=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "packed_sort or wide_top_digit or tiny_shapes" > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
bash $T/gpu_env_ab.sh $TAG 10e9 10 II_LIB_VARIANT=r4j - II_SEGHIST=0 II_SEGHIST=2 II_LIB_VARIANT=r4j && \
r7 mode1 II_NONE=1 && r7 mode0 II_SEGHIST=0 && r7 mode2 II_SEGHIST=2 && r7 r4j II_LIB_VARIANT=r4j && \
echo "== exchange timing" && timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 > $OUT/xchg.json 2> $OUT/xchg.err && tail -c 330 $OUT/xchg.json && \
echo "== exchange timing r4j" && II_LIB_VARIANT=r4j timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 > $OUT/xchg_r4j.json 2> $OUT/xchg_r4j.err && tail -c 330 $OUT/xchg_r4j.json
