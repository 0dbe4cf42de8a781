AB=nodeembedding-to-communityembedding_amd/csrc/build/ab
bash scripts/steps.sh r05e \
 "abc5|1100|AB_SECS=500 bash scripts/ab.sh r05e_c5 'python bench.py --nodes 10000000 --dim 256 --negative 10 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary' 1 base: w4:COME_LIB_PATH=$AB/libcome_c5w4.so"
