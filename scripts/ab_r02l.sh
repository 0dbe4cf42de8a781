set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/diag_tierc.py --variants sequential,hot_p1e-5,hot_p5e-6,hot_p3e-6 --hot-p 1e-5,5e-6,3e-6 > gpurun_out/r02l_diag.log 2>&1 || exit 1
for V in "--hot-p 1e-5" "--hot-p 5e-6" "--hot-p 3e-6"; do
  echo "== $V" >> gpurun_out/r02l_bench.log
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $V >> gpurun_out/r02l_bench.log 2>/dev/null || exit 1
done
