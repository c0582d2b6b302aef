#!/bin/bash
# one session: the 64-way merge-path partition and the launch-bounded wide MSD scatter — parity tests,
# then same-box A/B against the previous build (libii_nob.so) on the rank-7 share and the owner merge
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
r7() {  # r7 NAME ENV...
    local name=$1; shift
    echo "== rank 7 $name"
    env "$@" timeout -k 10 400 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 --no-cpu-baseline \
        --io-bytes 0 --no-verify > $OUT/r7_$name.log 2>&1 && tail -1 $OUT/r7_$name.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); p=d['phases_ms']; s=d['roofline_sort_phase']
print('value=%.1f ms/step=%.2f sort_phase=%.4f sort0=%.3f scat=%.3f ms_sort=%.3f ms_reduce=%.3f emit=%.3f' % (
 d['value'], d['ms_per_step'], s['frac'], s['first_pass']['ms'], d['roofline_sort']['ms_per_launch'], p['ms_sort'], p['ms_reduce'], p['emit_ms']))"
}
echo "== tests" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "owner_sort or logical_shards or two_ranks or cli_gpu or failed_owner or wide_top_digit or config5_shape or tiny_shapes" \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
r7 base II_NONE=1 && r7 nob II_LIB_VARIANT=nob && r7 base2 II_NONE=1 && \
echo "== exchange timing, one corpus" && timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 corpus > $OUT/xchg.json 2> $OUT/xchg.err && tail -c 330 $OUT/xchg.json && \
echo "== exchange timing, one corpus, nob" && II_LIB_VARIANT=nob timeout -k 10 300 python $T/exchange_timing.py 1.25e9 8 3 1 corpus > $OUT/xchg_nob.json 2> $OUT/xchg_nob.err && tail -c 330 $OUT/xchg_nob.json
