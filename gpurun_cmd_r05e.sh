AB=nodeembedding-to-communityembedding_amd/csrc/build/ab
bash scripts/steps.sh r05e \
 "replicas_o1|600|python -u scripts/tierc_replicas.py --fixture c2 --passes 4 --worlds 2,4,8 --periods 0 --combines owner --substeps 1,4,16,64 --out gpurun_out/r05e_tierc_replicas_c2_owner.json" \
 "tierc|600|python -u -m pytest tests/test_gpu_tierc.py -q -s -k '(multi_rank and not o1) or bench_launch or hogwild_c5 or default_period or benchmarked' --timeout 300 --timeout-method thread" \
 "abc5|1100|AB_SECS=500 bash scripts/ab.sh r05e_c5 'python bench.py --nodes 10000000 --dim 256 --negative 10 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary' 1 base: w4:COME_LIB_PATH=$AB/libcome_c5w4.so"
