#!/bin/bash
# one session: the one-launch import (a workgroup per source slice, batched loads) — exchange parity
# tests, then the owner-merge timing against libii_nob.so (per-source launches), alternated
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4q}
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
print('import %.3f owner sort %.3f map %.3f dict %.3f reduce %.3f' % (d['import'], d['owner_ms_sort'], d['owner_ms_map'], d['owner_ms_dict'], d['owner_ms_reduce']))"
}
echo "== tests" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "owner_sort or logical_shards or two_ranks or cli_gpu or failed_owner or tiny_shapes" \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
x base II_NONE=1 && x nob II_LIB_VARIANT=nob && x base2 II_NONE=1 && x nob2 II_LIB_VARIANT=nob
