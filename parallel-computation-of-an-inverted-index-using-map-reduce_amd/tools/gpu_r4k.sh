#!/bin/bash
# one session: tests of the fail-fast big-table probe, the rank-7 bench line, then SQ / TCC counter
# passes of the sort-phase kernels on the rank-7 share and on config3 (per-record costs side by side)
T=parallel-computation-of-an-inverted-index-using-map-reduce_amd/tools
TAG=${1:-r4k}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
RE="k_uniq_sweep|k_seg_hist|k_sort0_compact|k_onesweep_seg|k_msd_scatter|k_radix_scatter|k_tok_emit"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum"
echo "== tests" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "config5_shape or share7of8 or wide_top_digit or map_host or large_vocab or table_sized or tiny_shapes" \
    > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] && \
echo "== rank 7" && timeout -k 10 400 python bench.py --workload config5 --rank-share 7/8 --steps 5 --warmup 2 --no-cpu-baseline \
    --io-bytes 0 > $OUT/r7.log 2>&1 && tail -1 $OUT/r7.log | cut -c1-200 && \
echo "== pmc rank 7" && bash $T/gpu_pmc.sh $OUT/pmc_r7 "$RE" "$P1" "$P2" -- \
    python3 bench.py --workload config5 --rank-share 7/8 --steps 1 --warmup 0 --no-cpu-baseline --io-bytes 0 --no-verify && \
echo "== pmc config3" && bash $T/gpu_pmc.sh $OUT/pmc_c3 "$RE" "$P1" "$P2" -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --io-bytes 0 --no-verify
