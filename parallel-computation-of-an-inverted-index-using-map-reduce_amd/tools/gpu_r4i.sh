#!/bin/bash
# one session: the first-pass forms' parity tests, then same-box A/B of the paired first pass and the
# split first-pass output at config3, then the rank-7 share of configs[4] (packed since the wide digit)
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
r7() {  # r7 NAME ENV...
    local name=$1; shift
    echo "== rank 7 $name"
    env "$@" timeout -k 10 400 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 --no-cpu-baseline \
        --io-bytes 0 > $OUT/r7_$name.log 2>&1 && tail -1 $OUT/r7_$name.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); p=d['phases_ms']; s=d['roofline_sort_phase']
print('value=%.1f verified=%s packed=%s ms/step=%.2f sort_phase=%.4f sort0=%.3f ms_sort=%.3f ms_reduce=%.3f emit=%.3f' % (
 d['value'], d.get('verified'), d['counts'].get('sort_packed'), d['ms_per_step'], s['frac'], s['first_pass']['ms'], p['ms_sort'], p['ms_reduce'], p['emit_ms']))"
}
echo "== tests" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "first_pass_forms or sweep_two_tiles or packed_sort or tiny_shapes or owner_sort or logical_shards or export_after_reduce or two_ranks" > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
bash $T/gpu_env_ab.sh $TAG 10e9 10 - II_S0_HALF=1 II_S0_SPLIT=1 "II_S0_HALF=1 II_S0_SPLIT=1" II_SWEEP_TPW=2 - && \
r7 base II_NONE=1 && r7 split II_S0_SPLIT=1
[ $? = 0 ] && echo "== exchange timing" && timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 > $OUT/xchg.json 2> $OUT/xchg.err && tail -c 700 $OUT/xchg.json && \
echo "== rocprof exchange timing (G=8 owner import kernels)" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/xprof -o run -- \
    python3 $T/exchange_timing.py 1.25e9 8 1 1 > $OUT/xprof.log 2>&1 && echo "xprof ok"
