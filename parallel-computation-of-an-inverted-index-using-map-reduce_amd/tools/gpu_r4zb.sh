#!/bin/bash
# one session: the first pass's record-set dedup (k_sort0_compact<.., kHashD>) for small-file
# shares — the whole -m gpu suite, then the rank-7 share verified, and a same-box A/B against
# the epoch bitmap (II_S0_DEDUP=bitmap) on ranks 7 and 0
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4zb}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
share() {  # share R NAME ENV...
    local r=$1 name=$2; shift 2
    echo "== rank $r $name"
    env "$@" timeout -k 10 400 python bench.py --workload config5 --rank-share $r/8 --steps 5 --warmup 2 --no-cpu-baseline \
        --io-bytes 0 --no-verify > $OUT/r${r}_$name.log 2>&1 && tail -1 $OUT/r${r}_$name.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); p=d['phases_ms']; c=d['counts']
print('value=%.1f ms/step=%.2f emit=%.3f ms_sort=%.3f ms_reduce=%.3f sorted=%d pairs=%d' % (
 d['value'], d['ms_per_step'], p['emit_ms'], p['ms_sort'], p['ms_reduce'], c['sorted_records'], c['pairs']))"
}
echo "== pytest -m gpu" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
echo "== rank 7 verified" && timeout -k 10 500 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 \
    --no-cpu-baseline --io-bytes 0 > $OUT/r7_verified.log 2>&1 && tail -1 $OUT/r7_verified.log | cut -c1-200 && \
share 7 set II_NONE=1 && share 7 bitmap II_S0_DEDUP=bitmap && share 7 set2 II_NONE=1 && share 7 bitmap2 II_S0_DEDUP=bitmap && \
share 0 auto II_NONE=1 && share 0 set II_S0_DEDUP=set
