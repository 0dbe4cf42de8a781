set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/diag_tierc.py --no-oracle --repeat 8 --hot-p 5e-6 --waves 6144,4096 --variants hot_p5e-6_w6144,hot_p5e-6_w4096 > gpurun_out/r02ab_diag.log 2>&1 || exit 1
for V in "--opt max_waves=4096" "--opt max_waves=6144" ""; do
  echo "== [$V]" >> gpurun_out/r02ab_bench.log
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $V >> gpurun_out/r02ab_bench.log 2>/dev/null || exit 1
done
