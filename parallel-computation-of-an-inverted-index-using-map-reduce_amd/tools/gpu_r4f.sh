# one session: the exchange / merge / sort tests, owner-merge timing (working tree vs round 3),
# the default bench verified, the rank-7 share verified
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash $T/gpu_sel.sh $TAG "logical_shards or owner_sort or export_after_reduce or failed_owner or cli_gpu_counts or config5_shape or packed_sort_forms or tiny_shapes or two_ranks or map_host_matches" 0 && \
echo "== exchange timing base" && timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 > $OUT/xchg_base.json 2> $OUT/xchg_base.err && tail -c 1500 $OUT/xchg_base.json && \
echo "== exchange timing r3" && II_LIB_VARIANT=r3 timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 > $OUT/xchg_r3.json 2> $OUT/xchg_r3.err && tail -c 1500 $OUT/xchg_r3.json && \
echo "== bench rank 7" && timeout -k 10 400 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 --no-cpu-baseline --io-bytes 0 > $OUT/bench_r7.log 2>&1 && tail -1 $OUT/bench_r7.log | cut -c1-400
