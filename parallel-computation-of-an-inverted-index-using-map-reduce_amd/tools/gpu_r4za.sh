#!/bin/bash
# one session: K3 kFmap instances (the non-fmap one branch-free) — parity, rank-7 and
# config3 A/B against the HEAD build (libii_prev.so) twice, then the final profile
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4za}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
r7() {  # r7 NAME ENV...
    local name=$1; shift
    echo "== rank 7 $name"
    env "$@" timeout -k 10 400 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 --no-cpu-baseline \
        --io-bytes 0 --no-verify > $OUT/r7_$name.log 2>&1 && tail -1 $OUT/r7_$name.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); p=d['phases_ms']
print('value=%.1f ms/step=%.2f emit=%.3f resolve=%.3f ms_sort=%.3f ms_reduce=%.3f' % (
 d['value'], d['ms_per_step'], p['emit_ms'], p['resolve_ms'], p['ms_sort'], p['ms_reduce']))"
}
echo "== tests" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "bench_verify or config5_shape or global_ids or packed_sort or wide_top or logical_shards or export_after" \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
r7 base II_NONE=1 && r7 prev II_LIB_VARIANT=prev && \
bash $T/gpu_env_ab.sh $TAG 10e9 10 - II_LIB_VARIANT=prev - II_LIB_VARIANT=prev && \
bash $T/gpu_profile.sh ${TAG}_prof
