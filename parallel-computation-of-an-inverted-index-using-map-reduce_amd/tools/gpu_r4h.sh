#!/bin/bash
# one session: the sort / exchange / merge tests of this round's changes, then the owner-merge
# timing (working tree vs the round-3 library, libii_r3.so)
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4h}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "first_pass_forms or packed_sort or config5_shape or tiny_shapes or global_ids or bench_verify or logical_shards or owner_sort or export_after_reduce or failed_owner or two_ranks or map_host_matches" \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
echo "== exchange timing base" && timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 > $OUT/xchg_base.json 2> $OUT/xchg_base.err && tail -c 1500 $OUT/xchg_base.json && \
echo "== exchange timing r3" && II_LIB_VARIANT=r3 timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 > $OUT/xchg_r3.json 2> $OUT/xchg_r3.err && tail -c 1500 $OUT/xchg_r3.json
