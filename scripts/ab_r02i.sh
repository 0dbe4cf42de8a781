set -o pipefail
mkdir -p gpurun_out
for V in "" "--opt o2_blocks_per_cu=7" "W8 --opt o2_blocks_per_cu=8" "W8 --opt o2_blocks_per_cu=7" "W8"; do
  echo "== $V" >> gpurun_out/r02i_bench.log
  if [[ "$V" == W8* ]]; then export COME_LIB_PATH=$PWD/nodeembedding-to-communityembedding_amd/libcome_w8.so; V=${V#W8}; else unset COME_LIB_PATH; fi
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $V >> gpurun_out/r02i_bench.log 2>/dev/null || exit 1
done
