set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02ah_bench.json 2>/dev/null || exit 1
timeout -k 10 300 python -u scripts/diag_tierc.py --nodes 1000000 --walks 16000 --repeat 2 --hot-p 5e-6 --variants stream_hot_p5e-6 > gpurun_out/r02ah_diag.log 2>&1 || exit 1
timeout -k 10 900 python -u scripts/tierc_scale.py --out gpurun_out/r02ah_tierc_scale.json > gpurun_out/r02ah.log 2>&1 || exit 1
