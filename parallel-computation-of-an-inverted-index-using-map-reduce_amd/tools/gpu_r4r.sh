#!/bin/bash
# one session: the single-launch small scan through the whole GPU suite, then the owner-merge timing and
# config3 against the previous build (libii_prev.so), and config3 at a 9 / 10-bit top digit
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
x() {  # x NAME ENV...
    local name=$1; shift
    echo "== exchange timing $name"
    env "$@" timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 corpus > $OUT/xchg_$name.json 2> $OUT/xchg_$name.err && \
    python3 -c "
import json,sys
d=json.load(open('$OUT/xchg_$name.json'))['phases_ms_all_shards']['per_shard_ms']
print(' '.join('%s %.3f' % (k, d[k]) for k in ('map','reduce_local','plan_export','import','order_format','owner_ms_map','owner_ms_dict','owner_ms_sort','owner_ms_reduce')))"
}
echo "== pytest -m gpu" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
x base II_NONE=1 && x prev II_LIB_VARIANT=prev && \
bash $T/gpu_env_ab.sh $TAG 10e9 10 - II_LIB_VARIANT=prev II_PACKED_M=9 II_PACKED_M=10 -
