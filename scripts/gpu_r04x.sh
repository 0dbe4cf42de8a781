#!/bin/bash
# Round 3 (driver): k_community16 (community_async = 2: 16x16x4 MFMAs, one row tile per wavefront)
# -- community parity tests, then C4 A/B against k_community_async (= 1), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c4.py -m gpu -v -k "community" \
  --timeout 200 --timeout-method thread > gpurun_out/r04x_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r04x_pytest.log | tail -12
[ $PYTEST_RC -eq 0 ] || exit $PYTEST_RC
for R in 1 2 1 2; do
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt community_async=$R > gpurun_out/r04x_c4_$R.json 2> gpurun_out/r04x_c4.err \
    || { echo "c4 failed"; tail -20 gpurun_out/r04x_c4.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04x_c4_$R.json'));r=j['roofline'];print('comm=$R', j['value'], j['ms_per_step'], r.get('frac'), r.get('achieved'), r.get('avg_kernel_ms'))"
done
exit 0
