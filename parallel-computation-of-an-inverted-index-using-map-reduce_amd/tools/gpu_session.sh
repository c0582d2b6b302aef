#!/bin/bash
# gpu_session.sh TAG STEP... — one GPU-box session, the steps in order, each
# GPU step under its own time limit; the first failure ends the session (no
# retries).  Results land in gpurun_out/TAG/.  Steps:
#   tests                  the whole -m gpu suite
#   tests:EXPR             the -m gpu tests selected by pytest -k EXPR
#   bench                  the default bench line (CPU baselines, io legs)
#   quick[:ARGS]           a bench line without CPU baselines / io legs (+ARGS)
#   prof[:ARGS]            rocprofv3 kernel statistics + trace of a quick bench (+ARGS)
#   prof5r7[:NAME[:ENV=V,...]]  the same on configs[4]'s rank-7 share, under extra environment variables
#   pmc                    the PMC traffic passes (profiles/pmc_traffic.py) + summary
#   ab:VARIANTS            same-box A/B at configs[2]: base (libii.so) and libii_<v>.so
#                          (tools/build_variant.sh / build_rev.sh); VARIANTS comma-separated
#   ab5r7:VARIANTS         the same on configs[4]'s rank-7 share
#   env:NAME:ENV=V,...     a quick bench line under extra environment variables
#   xchg[:G]               tools/exchange_timing.py 1.25e9 G 3 1 corpus (G = 8), kernel trace
#   sortbench              tools/sort_bench (onesweep pass vs copy vs rocPRIM)
#   listpmc                rocprofv3 -L (the counters of this GPU)
#   sq[:REGEX[:ARGS]]      SQ counter passes (tools/gpu_pmc.sh) over a short bench (+ARGS), kernels
#                          matching REGEX (default k_tok_emit|k_sort0_compact)
# Example:  gpu_session.sh r5a tests prof sortbench
set -o pipefail
TAG=${1:?tag}
shift
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
T="$ROOT/parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools"
PKG="$ROOT/parallel-computation-of-an-inverted-index-using-map-reduce_amd"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
QB="--steps 10 --warmup 2 --no-cpu-baseline --io-bytes 0"

summ() {  # one bench line -> a short summary
    tail -1 "$1" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); p=d['phases_ms']; s=d['roofline_sort_phase']
print('%s value=%.1f ms/step=%.2f verified=%s emit=%.3f sort0=%.3f ms_sort=%.3f ms_reduce=%.3f fmt=%.3f sort_frac=%.4f' % (
 '$2', d['value'], d['ms_per_step'], d['verified'], p['emit_ms'], s['first_pass']['ms'], p['ms_sort'],
 p['ms_reduce'], p['ms_format'], s['frac']))"
}

step() {
    local s=$1 name=${1%%:*} arg=""
    [ "$s" != "$name" ] && arg=${s#*:}
    echo "== $s"
    case $name in
    tests)
        local k=()
        [ -n "$arg" ] && k=(-k "$arg")
        timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v "${k[@]}" --timeout 300 --timeout-method thread \
            > "$OUT/pytest_gpu.log" 2>&1
        local rc=$?
        tail -3 "$OUT/pytest_gpu.log"
        return $rc ;;
    bench)
        timeout -k 10 600 python bench.py > "$OUT/bench.log" 2>&1 && summ "$OUT/bench.log" bench ;;
    quick)
        # shellcheck disable=SC2086
        timeout -k 10 300 python bench.py $QB $arg > "$OUT/quick.log" 2>&1 && summ "$OUT/quick.log" quick ;;
    prof)
        # shellcheck disable=SC2086
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
            python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify $arg \
            > "$OUT/prof.log" 2>&1 && echo "rocprof ok" ;;
    prof5r7)
        # rocprofv3 kernel statistics of configs[4]'s rank-7 share; arg NAME[:ENV=V,...]
        local nm=${arg%%:*} ev=""
        [ "$arg" != "$nm" ] && ev=${arg#*:}
        # shellcheck disable=SC2086
        ( [ -n "$ev" ] && export ${ev//,/ }
          timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof5r7_${nm:-base}" -o run -- \
            python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify --workload config5 \
            --rank-share 7/8 > "$OUT/prof5r7_${nm:-base}.log" 2>&1 ) && echo "rocprof ok" ;;
    pmc)
        timeout -k 10 600 python3 profiles/pmc_traffic.py run "$OUT/pmc" --steps 3 --warmup 1 --no-cpu-baseline \
            --io-bytes 0 --no-verify && python3 profiles/pmc_traffic.py summarize "$OUT/pmc" > "$OUT/pmc_traffic.json" &&
            echo "pmc ok" ;;
    ab)
        bash "$T/gpu_ab.sh" "$TAG/ab3" 10000000000 10 base ${arg//,/ } ;;
    ab5r7)
        AB_ARGS="--workload config5 --rank-share 7/8" bash "$T/gpu_ab.sh" "$TAG/ab5r7" - 5 base ${arg//,/ } ;;
    env)
        local nm=${arg%%:*} ev=${arg#*:}
        # shellcheck disable=SC2086
        env ${ev//,/ } timeout -k 10 300 python bench.py $QB > "$OUT/env_$nm.log" 2>&1 && summ "$OUT/env_$nm.log" "$nm" ;;
    xchg)
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/xchg" -o run -- \
            python3 "$T/exchange_timing.py" 1.25e9 "${arg:-8}" 3 1 corpus > "$OUT/xchg.log" 2>&1 && tail -1 "$OUT/xchg.log" ;;
    sortbench)
        timeout -k 10 300 "$PKG/sort_bench" > "$OUT/sort_bench.log" 2>&1 && cat "$OUT/sort_bench.log" ;;
    sq)
        local rx=${arg%%:*} bargs=""
        [ "$arg" != "$rx" ] && bargs=${arg#*:}
        # shellcheck disable=SC2086
        bash "$T/gpu_pmc.sh" "$OUT/sq" "${rx:-k_tok_emit|k_sort0_compact}" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT" \
            "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_LDS_ATOMIC" \
            "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_BUBBLE_sum" \
            -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --io-bytes 0 --no-verify $bargs &&
            python3 "$T/sq_summary.py" "$OUT/sq" > "$OUT/sq_summary.txt" && echo "sq ok" ;;
    listpmc)
        timeout -k 10 120 rocprofv3 -L > "$OUT/rocprofv3_L.txt" 2>&1 && echo "listed $(wc -l < "$OUT/rocprofv3_L.txt") lines" ;;
    *)
        echo "unknown step $s"; return 2 ;;
    esac
}

for s in "$@"; do
    step "$s" || { echo "step $s failed ($?)"; exit 1; }
done
echo "session $TAG done"
