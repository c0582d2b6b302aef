#!/bin/bash
# one session: a third batched probe round of the first pass's record set (libii_r3.so, built
# from a patched copy of the sources) against the tree's build, same box, rank-7 share
TAG=${1:-r4zi}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
share() {  # share R NAME ENV...
    local r=$1 name=$2; shift 2
    echo "== rank $r $name"
    env "$@" timeout -k 10 400 python bench.py --workload config5 --rank-share $r/8 --steps 5 --warmup 2 --no-cpu-baseline \
        --io-bytes 0 --no-verify > $OUT/r${r}_$name.log 2>&1 && tail -1 $OUT/r${r}_$name.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); p=d['phases_ms']; c=d['counts']; s=d['roofline_sort_phase']
print('value=%.1f ms/step=%.2f emit=%.3f first=%.3f ms_sort=%.3f ms_reduce=%.3f sorted=%d' % (
 d['value'], d['ms_per_step'], p['emit_ms'], s['first_pass']['ms'], p['ms_sort'], p['ms_reduce'], c['sorted_records']))"
}
echo "== rank 7 r3 verified" && II_LIB_VARIANT=r3 timeout -k 10 500 python bench.py --workload config5 --rank-share 7/8 \
    --steps 3 --warmup 1 --no-cpu-baseline --io-bytes 0 > $OUT/r7_r3_verified.log 2>&1 && \
tail -1 $OUT/r7_r3_verified.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'])" && \
share 7 base II_NONE=1 && share 7 r3 II_LIB_VARIANT=r3 && share 7 base2 II_NONE=1 && share 7 r3_2 II_LIB_VARIANT=r3
