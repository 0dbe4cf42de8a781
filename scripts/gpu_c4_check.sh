# GMM GPU tests + C4 bench (tag in $1)
set -o pipefail
mkdir -p gpurun_out
T=${1:-c4}
timeout -k 10 400 python -u -m pytest tests/test_gpu_gmm.py -q -x --timeout 300 --timeout-method thread > gpurun_out/${T}_gmm.log 2>&1 || { tail -30 gpurun_out/${T}_gmm.log; exit 1; }
timeout -k 10 200 python bench_aux.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c4.json 2> gpurun_out/${T}_c4.err || exit 1
