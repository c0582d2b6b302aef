set -o pipefail
mkdir -p gpurun_out/r3g
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli_multi.py tests/test_gpu_dist.py tests/test_gpu_parity.py -k "cli or dist or shard or tiny" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3g/pytest.log 2>&1 || { tail -30 gpurun_out/r3g/pytest.log; exit 1; }
tail -2 gpurun_out/r3g/pytest.log
cd parallel-computation-of-an-inverted-index-using-map-reduce_amd
timeout -k 10 300 python tools/exchange_timing.py 1.25e9 8 3 1 > ../gpurun_out/r3g/xchg_merge.json 2>&1 && cat ../gpurun_out/r3g/xchg_merge.json
II_IMPORT_ID_SORT=1 timeout -k 10 300 python tools/exchange_timing.py 1.25e9 8 3 1 > ../gpurun_out/r3g/xchg_sort.json 2>&1 && cat ../gpurun_out/r3g/xchg_sort.json
bash tools/gpu_pmc.sh ../gpurun_out/r3g/pmc "k_emit_variant|k_tok_count|k_read_only" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY" -- ./k1_ablate 1000000000 1000 1000000
