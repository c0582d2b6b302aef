#!/bin/bash
# one session for the round's last build (record set, single entries, two batched rounds): the whole
# -m gpu suite, smoke(), the final
# profile (bench line, rocprof kernel stats, PMC traffic), the default bench line again with that
# PMC summary in profiles/, then the N > 1 lines
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4zh}
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
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log && \
bash $T/gpu_profile.sh ${TAG}_prof && \
cp gpurun_out/${TAG}_prof/pmc_traffic.json profiles/${TAG}_onbox_pmc_traffic.json && \
echo "== bench" && timeout -k 10 500 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-200 && \
bash $T/gpu_multi.sh $TAG
