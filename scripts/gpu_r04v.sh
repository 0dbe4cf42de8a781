#!/bin/bash
# Round 3 (driver): k_gmm_resp16t wave-shape variants -- GMM tests (bit-identity across shapes,
# FULL launches), then C4 A/B: gmm_resp16 = 16 + i over VT {0, 2, 8, 10, 26}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gmm.py tests/test_gpu_c4.py -m gpu -v \
  --timeout 200 --timeout-method thread > gpurun_out/r04v_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r04v_pytest.log | tail -12
[ $PYTEST_RC -eq 0 ] || exit $PYTEST_RC
for P in 1 2; do
for R in 16 17 18 19 20; do
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_resp16=$R > gpurun_out/r04v_c4_$R.json 2> gpurun_out/r04v_c4.err \
    || { echo "c4 failed"; tail -20 gpurun_out/r04v_c4.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04v_c4_$R.json'));c=j['config'];print('r16=$R', round(c['gmm_resp_ms'],3), round(c['gmm_resp_tflops_executed'],1))"
done
done
exit 0
