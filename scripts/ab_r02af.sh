set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_tierc.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r02af_tierc.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02af_bench.json 2>/dev/null || exit 1
