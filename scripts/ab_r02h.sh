set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s -k "tierc" > gpurun_out/r02h_tierc.log 2>&1; echo "pytest rc=$?" >> gpurun_out/r02h_tierc.log
for V in "--hot-p 0" "" "--packed-table" "--opt o2_blocks_per_cu=5" "--opt o2_blocks_per_cu=4" "--opt o2_blocks_per_cu=8" "--opt o2_kernel=1"; do
  echo "== $V" >> gpurun_out/r02h_bench.log
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $V >> gpurun_out/r02h_bench.log 2>/dev/null || exit 1
done
