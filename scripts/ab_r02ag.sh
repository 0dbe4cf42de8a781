set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/diag_tierc.py --nodes 1000000 --walks 16000 --repeat 2 --hot-p 5e-6,1e-6,1e-7,1e-9 --variants stream_hot_p5e-6,stream_hot_p1e-6,stream_hot_p1e-7,stream_hot_p1e-9,direct_hot_p5e-6,direct_hot_p1e-9 > gpurun_out/r02ag_diag.log 2>&1 || exit 1
for V in "--hot-p 1e-7" "--hot-p 1e-9"; do
  echo "== [$V]" >> gpurun_out/r02ag_bench.log
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $V >> gpurun_out/r02ag_bench.log 2>/dev/null || exit 1
done
