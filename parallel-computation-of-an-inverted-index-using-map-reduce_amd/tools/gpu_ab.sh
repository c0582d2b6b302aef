#!/bin/bash
# gpu_ab.sh — A/B of kernel variants on one GPU box: bench.py once per
# libii_<variant>.so (built beforehand on the CPU side with extra -D flags,
# tools/build_variant.sh), each under its own time limit; the first failure
# ends the session.
#   tools/gpu_ab.sh TAG BYTES STEPS VARIANT...   ("base" = libii.so)
# BYTES = "-": the workload comes from $AB_ARGS instead (e.g. "--workload config5 --rank-share 0/8").
set -o pipefail
TAG=$1; BYTES=$2; STEPS=$3; shift 3
if [ "$BYTES" = "-" ]; then WL="$AB_ARGS"; else WL="--bytes $BYTES"; fi
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT" || exit 1
for v in "$@"; do
    echo "== $v"
    if [ "$v" = "base" ]; then
        timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 2 $WL --no-cpu-baseline --io-bytes 0 \
            > "$OUT/bench_$v.log" 2>&1 || exit $?
    else
        II_LIB_VARIANT=$v timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 2 $WL \
            --no-cpu-baseline --io-bytes 0 > "$OUT/bench_$v.log" 2>&1 || exit $?
    fi
    tail -1 "$OUT/bench_$v.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); p=d['phases_ms']; s=d['roofline_sort_phase']
print('%s value=%.1f ms/step=%.2f sort_phase=%.4f sort0=%.3f scatter=%.3f emit=%.3f resolve=%.3f ms_sort=%.3f ms_reduce=%.3f ms_map=%.3f fmt=%.3f' % (
 '$v', d['value'], d['ms_per_step'], s['frac'], s['first_pass']['ms'], d['roofline_sort']['ms_per_launch'],
 p['emit_ms'], p['resolve_ms'], p['ms_sort'], p['ms_reduce'], p['ms_map'], p['ms_format']))"
done
