#!/bin/bash
# one session: sort / exchange tests of the cleaned-up build, owner-merge timing with the
# persistent merge tiles, a config3 bench line, and the rank-7 share's kernel statistics
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4j}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "wide_top_digit or packed_sort or tiny_shapes or owner_sort or logical_shards or export_after_reduce or two_ranks or config5_shape or map_host or failed" \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
echo "== exchange timing" && timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 > $OUT/xchg.json 2> $OUT/xchg.err && tail -c 700 $OUT/xchg.json && \
echo "== bench config3" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --io-bytes 0 > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-200 && \
echo "== rocprof rank 7" && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r7prof -o run -- \
    python3 bench.py --workload config5 --rank-share 7/8 --steps 3 --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify > $OUT/r7prof.log 2>&1 && echo "r7prof ok"
