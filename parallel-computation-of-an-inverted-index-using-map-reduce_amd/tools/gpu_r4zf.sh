#!/bin/bash
# one session: the record set probed by aligned entry pairs (two rounds) — parity selection, then same-box
# A/B against the HEAD build (libii_prev.so) on the rank-7 share
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4zf}
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
echo "== pytest -m gpu" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "record_set or random_corpora or wide_top or global_ids" > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
share 7 new II_NONE=1 && share 7 prev II_LIB_VARIANT=prev && share 7 new2 II_NONE=1 && share 7 prev2 II_LIB_VARIANT=prev && \
share 0 auto II_NONE=1 && share 0 prev II_LIB_VARIANT=prev
