bash scripts/steps.sh r05a \
 "gmm|600|python -u -m pytest tests/test_gpu_gmm.py tests/test_gpu_c4.py -x -q --timeout 240 --timeout-method thread && python -u -m pytest tests/test_gpu_parity.py -x -q -k 'community or gmm' --timeout 240 --timeout-method thread" \
 "replicas|900|python -u scripts/tierc_replicas.py --fixture c3_1m --worlds 1,2,4,8 --periods 131072,32768,8192 --combines pick,hot_pick,touched_mean --out gpurun_out/r05a_tierc_replicas_c3_1m.json" \
 "counters|90|cd /tmp && timeout -s KILL 60 rocprofv3 -L" \
 "pmc01|600|TAG=r05a_pmc_o1_lr0.1 KERNEL=sgns_o1 CMD='bench_aux.py --workload c2 --steps 4 --warmup 1 --no-cpu-baseline --lr 0.1' bash scripts/pmc.sh FETCH_SIZE WRITE_SIZE 'SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES' 'TCC_HIT_sum TCC_MISS_sum'" \
 "pmc02|600|TAG=r05a_pmc_o1_lr0.2 KERNEL=sgns_o1 CMD='bench_aux.py --workload c2 --steps 4 --warmup 1 --no-cpu-baseline --lr 0.2' bash scripts/pmc.sh FETCH_SIZE WRITE_SIZE 'SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES' 'TCC_HIT_sum TCC_MISS_sum'"
