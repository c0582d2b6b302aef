#!/bin/bash
# gpu_env_ab.sh TAG BYTES STEPS "ENV=VAL ..." ... — bench.py once per environment
# setting ("-" = none), each under its own time limit; first failure ends it.
set -o pipefail
TAG=$1; BYTES=$2; STEPS=$3; shift 3
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT" || exit 1
i=0
for e in "$@"; do
    i=$((i + 1))
    echo "== $e"
    if [ "$e" = "-" ]; then e=""; fi
    # shellcheck disable=SC2086
    env $e timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 2 --bytes "$BYTES" --no-cpu-baseline \
        --io-bytes 0 > "$OUT/bench_$i.log" 2>&1 || exit $?
    tail -1 "$OUT/bench_$i.log" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); p=d['phases_ms']; s=d['roofline_sort_phase']
print('value=%.1f ms/step=%.2f sort_phase=%.4f sort0=%.3f scatter=%.3f emit=%.3f resolve=%.3f ms_sort=%.3f ms_reduce=%.3f ms_map=%.3f dict=%.3f fmt=%.3f cap=%d' % (
 d['value'], d['ms_per_step'], s['frac'], s['first_pass']['ms'], d['roofline_sort']['ms_per_launch'],
 p['emit_ms'], p['resolve_ms'], p['ms_sort'], p['ms_reduce'], p['ms_map'], p['ms_dict'], p['ms_format'], d['counts']['table_cap']))"
done
