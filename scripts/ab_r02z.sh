set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/diag_tierc.py --no-oracle --repeat 5 --hot-p 5e-6,2e-6,1e-6 --waves 4096,2048 --variants hot_p5e-6,hot_p2e-6,hot_p1e-6,hot_p5e-6_w4096,hot_p5e-6_w2048,direct_fresh_atomic > gpurun_out/r02z_diag.log 2>&1 || exit 1
for V in "--hot-p 2e-6" "--hot-p 1e-6"; do
  echo "== $V" >> gpurun_out/r02z_bench.log
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $V >> gpurun_out/r02z_bench.log 2>/dev/null || exit 1
done
