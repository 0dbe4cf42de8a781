set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gmm.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r02y_gmm.log 2>&1 || { tail -30 gpurun_out/r02y_gmm.log; exit 1; }
for v in "" "--opt gmm_cov_async=2" "" "--opt gmm_cov_async=2"; do
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline $v > gpurun_out/ab_c4.json 2>/dev/null || exit 1
  echo "variant [$v]: $(python -c "import json;d=json.load(open('gpurun_out/ab_c4.json'));c=d['config'];print(c['gmm_scatter_ms'], c['gmm_em_iteration_ms'])")" >> gpurun_out/r02y_ab.log
done
