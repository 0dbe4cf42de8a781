#!/bin/bash
# Round 3 (driver): k_gmm_cov16<W=1> (gmm_cov_async = 4: 8 MFMA + 4 staging wavefronts, 4 MFMA
# waves per SIMD) -- scatter tests, then C4 A/B against k_gmm_cov16 (= 3), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gmm.py tests/test_gpu_c4.py -m gpu -v -k "scatter or em" \
  --timeout 200 --timeout-method thread > gpurun_out/r04y_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r04y_pytest.log | tail -12
[ $PYTEST_RC -eq 0 ] || exit $PYTEST_RC
for R in 3 4 3 4; do
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_cov_async=$R > gpurun_out/r04y_c4_$R.json 2> gpurun_out/r04y_c4.err \
    || { echo "c4 failed"; tail -20 gpurun_out/r04y_c4.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04y_c4_$R.json'));c=j['config'];print('cov=$R', c['gmm_scatter_kernel'], round(c['gmm_scatter_ms'],3), round(c['gmm_scatter_tflops_executed'],1), 'em', round(c['gmm_em_iteration_ms'],2), 'comm', round(j['ms_per_step'],3))"
done
exit 0
