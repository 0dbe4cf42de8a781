#!/bin/bash
# Round 3 (driver): the M-step scatter on 16x16x4 tiles (gmm_cov_async = 3, k_gmm_cov16) -- tests,
# then C4 A/B against k_gmm_cov_async (= 1), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_gmm.py -m gpu -v -k "scatter" --timeout 200 \
  --timeout-method thread > gpurun_out/r04m_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r04m_pytest.log | tail -12
[ $PYTEST_RC -eq 0 ] || exit $PYTEST_RC
I=0
for OPT in 1 3 1 3; do
  I=$((I+1))
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_cov_async=$OPT > gpurun_out/r04m_c4_${OPT}_$I.json 2> gpurun_out/r04m_c4_$I.err \
    || { echo "c4 failed"; tail -20 gpurun_out/r04m_c4_$I.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04m_c4_${OPT}_$I.json'));c=j['config'];print('cov=$OPT', {k:(round(c[k],3) if isinstance(c[k],float) else c[k]) for k in c if k.startswith('gmm_sc') or k.startswith('gmm_em')})"
done
