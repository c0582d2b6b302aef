#!/bin/bash
# gpu_xchg_ab.sh TAG — the owners' merge of interleaved sources at G = 2, 4, 8 (10 GB in total):
# k_merge_ids (default) against the id + word radix passes (II_IMPORT_ID_SORT=1), tools/exchange_timing.py.
set -o pipefail
TAG=${1:-xchg}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT/parallel-computation-of-an-inverted-index-using-map-reduce_amd" || exit 1
for cfg in "5e9 2" "2.5e9 4" "1.25e9 8"; do
    set -- $cfg
    timeout -k 10 300 python tools/exchange_timing.py "$1" "$2" 3 1 > "$OUT/merge_G$2.json" 2>&1 || exit $?
    II_IMPORT_ID_SORT=1 timeout -k 10 300 python tools/exchange_timing.py "$1" "$2" 3 1 > "$OUT/sort_G$2.json" 2>&1 || exit $?
    python3 -c "
import json,sys
for f in ['$OUT/merge_G$2.json','$OUT/sort_G$2.json']:
    d=json.loads(open(f).read().strip().split('\n')[-1]); p=d['phases_ms_all_shards']['per_shard_ms']
    print(f.split('/')[-1], 'import', p['import'], 'owner_sort', p['owner_ms_sort'], 'map', p['map'], 'reduce_local', p['reduce_local'])"
done
