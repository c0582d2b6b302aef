#!/bin/bash
# one session: export straight from word-id order (k_export_pairs_wid) — the exchange tests, then the
# G = 8 phase timing over one corpus against the previous build (libii_prev.so), alternated
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4u}
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
print(' '.join('%s %.3f' % (k, d[k]) for k in ('map','reduce_local','plan_export','exchange_copies','import','order_format')))"
}
echo "== tests" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "owner_sort or logical_shards or two_ranks or cli or export or balanced or tiny_shapes or letter" \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
x base II_NONE=1 && x prev II_LIB_VARIANT=prev && x base2 II_NONE=1 && x prev2 II_LIB_VARIANT=prev
