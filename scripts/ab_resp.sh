# GMM tests with the current library, then C4 bench: current vs a saved previous build (COME_LIB_PATH)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gmm.py -q -x --timeout 300 --timeout-method thread > gpurun_out/resp_gmm.log 2>&1 || { tail -30 gpurun_out/resp_gmm.log; exit 1; }
for v in cur prev cur prev; do
  if [ $v = prev ]; then export COME_LIB_PATH=$PWD/gpurun_ab_libcome_prev.so; else unset COME_LIB_PATH; fi
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_c4.json 2>/dev/null || exit 1
  echo "$v: $(python -c "import json;d=json.load(open('gpurun_out/ab_c4.json'));c=d['config'];print(c['gmm_resp_ms'], c['gmm_scatter_ms'], c['gmm_em_iteration_ms'])")" >> gpurun_out/resp_ab.log
done
