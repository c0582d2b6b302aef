#!/bin/bash
# one session: where the first pass's record set stops paying — configs[4] shares 3..6 with the
# dedup forced each way (II_S0_DEDUP), same box; the tree's build
TAG=${1:-r4zj}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
share() {  # share R NAME ENV...
    local r=$1 name=$2; shift 2
    echo "== rank $r $name"
    env "$@" timeout -k 10 400 python bench.py --workload config5 --rank-share $r/8 --steps 4 --warmup 1 --no-cpu-baseline \
        --io-bytes 0 --no-verify > $OUT/r${r}_$name.log 2>&1 && tail -1 $OUT/r${r}_$name.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); p=d['phases_ms']; c=d['counts']; s=d['roofline_sort_phase']
print('value=%.1f ms/step=%.2f first=%.3f ms_sort=%.3f ms_reduce=%.3f tokens=%d files=%d tok/file=%.0f sorted=%d pairs=%d' % (
 d['value'], d['ms_per_step'], s['first_pass']['ms'], p['ms_sort'], p['ms_reduce'], c['tokens'], c['files'], c['tokens']/c['files'], c['sorted_records'], c['pairs']))"
}
share 6 set II_S0_DEDUP=set && share 6 bitmap II_S0_DEDUP=bitmap && \
share 5 set II_S0_DEDUP=set && share 5 bitmap II_S0_DEDUP=bitmap && \
share 4 set II_S0_DEDUP=set && share 4 bitmap II_S0_DEDUP=bitmap && \
share 3 set II_S0_DEDUP=set && share 3 bitmap II_S0_DEDUP=bitmap
