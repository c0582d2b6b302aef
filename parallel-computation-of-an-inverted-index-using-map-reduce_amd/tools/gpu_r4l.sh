#!/bin/bash
# one session: parity of K3's threshold posting bytes, the wave-aggregated seg_hist and the one-launch
# import, then the rank-7 and config3 bench lines and the owner-merge timing
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4l}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "bench_verify or packed_sort or global_ids or wide_top_digit or config5_shape or logical_shards or owner_sort or two_ranks or tiny_shapes or map_host or export_after" \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
echo "== rank 7" && timeout -k 10 400 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 --no-cpu-baseline \
    --io-bytes 0 > $OUT/r7.log 2>&1 && tail -1 $OUT/r7.log | cut -c1-120 && \
echo "== config3" && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --io-bytes 0 > $OUT/c3.log 2>&1 && tail -1 $OUT/c3.log | cut -c1-120 && \
echo "== exchange timing" && timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 > $OUT/xchg.json 2> $OUT/xchg.err && tail -c 500 $OUT/xchg.json && \
echo "== rocprof rank 7" && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r7prof -o run -- \
    python3 bench.py --workload config5 --rank-share 7/8 --steps 3 --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify > $OUT/r7prof.log 2>&1 && echo "r7prof ok"
