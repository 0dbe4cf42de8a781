#!/bin/bash
# Round 3 (driver), seventh pass: the 16x16x4 E-step kernel (k_gmm_resp16) -- tests, then C4 A/B
# against k_gmm_resp_mfma, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gmm.py -m gpu -v -k "estep" \
  --timeout 120 --timeout-method thread > gpurun_out/r04g_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r04g_pytest.log | tail -12
[ $PYTEST_RC -eq 0 ] || exit $PYTEST_RC
I=0
for OPT in 0 1 0 1; do
  I=$((I+1))
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_resp16=$OPT > gpurun_out/r04g_c4_r16_${OPT}_$I.json 2> gpurun_out/r04g_c4_$I.err \
    || { echo "c4 r16=$OPT failed"; tail -20 gpurun_out/r04g_c4_$I.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04g_c4_r16_${OPT}_$I.json'));c=j['config'];print('r16=$OPT', {k:round(c[k],3) for k in c if k.startswith('gmm')})"
done
