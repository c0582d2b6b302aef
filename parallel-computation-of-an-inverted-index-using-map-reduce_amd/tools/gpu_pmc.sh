#!/bin/bash
# gpu_pmc.sh — rocprofv3 counter passes over one command, one pass per counter
# group (rocprofv3 does not split counters over passes), each under its own
# hard time limit.  A pass that fails quickly (unknown counter name) does not
# stop the others; a pass that hits its time limit ends the session.
#   tools/gpu_pmc.sh OUT_DIR KERNEL_REGEX "PASS1 COUNTERS" ["PASS2 COUNTERS" ...] -- CMD ARGS...
set -o pipefail
OUT=$1; REGEX=$2; shift 2
PASSES=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do PASSES+=("$1"); shift; done
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1
i=0
for ctrs in "${PASSES[@]}"; do
    i=$((i + 1))
    echo "== pass $i: $ctrs"
    # shellcheck disable=SC2086
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "$REGEX" --output-format csv \
        -d "$OUT/pass$i" -o run -- "$@" > "$OUT/pass$i.log" 2>&1
    rc=$?
    tail -2 "$OUT/pass$i.log"
    if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "pass $i ended with $rc: stopping"
        exit $rc
    fi
done
exit 0
