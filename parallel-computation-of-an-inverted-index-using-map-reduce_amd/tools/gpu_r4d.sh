# one session: parity selection, bit-width A/B at configs[2], rank-7 share vs round 3, kernel stats
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4e}
bash $T/gpu_sel.sh $TAG "map_host_matches or tiny_shapes or packed_sort_forms or config5_shape or zipf_medium or random_corpora or large_vocab or global_ids" 0 && \
bash $T/gpu_env_ab.sh $TAG/env 10000000000 10 - "II_SUB_BITS=7" "II_MSD1_BITS=7 II_SUB_BITS=7" && \
AB_ARGS="--workload config5 --rank-share 7/8" bash $T/gpu_ab.sh "$TAG/ab5r7" - 5 base r3 && \
mkdir -p gpurun_out/$TAG && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- \
    python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify > gpurun_out/$TAG/prof.log 2>&1 && echo rocprof ok
