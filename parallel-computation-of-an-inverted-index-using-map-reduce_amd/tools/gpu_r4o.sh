#!/bin/bash
# one session: the 8-bit MSD in k_msd_scatter (II_MSD256=1) against k_radix_scatter<kPack> at config3,
# then the owner-merge timing with the G shards cut from ONE corpus (bench.py's layout), and its kernels
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests (II_MSD256=1)" && \
II_MSD256=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "packed_sort or tiny_shapes or global_ids" > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
bash $T/gpu_env_ab.sh $TAG 10e9 10 - II_MSD256=1 - II_MSD256=1 && \
echo "== exchange timing, one corpus" && timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 corpus > $OUT/xchg.json 2> $OUT/xchg.err && tail -c 400 $OUT/xchg.json && \
echo "== rocprof exchange timing, one corpus" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/xprof -o run -- \
    python3 $T/exchange_timing.py 1.25e9 8 1 1 corpus > $OUT/xprof.log 2>&1 && echo "xprof ok"
