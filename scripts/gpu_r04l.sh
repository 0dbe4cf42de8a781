#!/bin/bash
# Round 3 (driver): the packed one-barrier E-step (gmm_resp16 = 2, k_gmm_resp16t) -- tests and A/B
# vs k_gmm_resp16; the single-launch tier C at the bench's 1M-walk launch; C2 hot/cold x lr.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_gmm.py -m gpu -v -k "estep" --timeout 200 \
  --timeout-method thread > gpurun_out/r04l_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r04l_pytest.log | tail -12
[ $PYTEST_RC -eq 0 ] || exit $PYTEST_RC
I=0
for OPT in 1 2 1 2; do
  I=$((I+1))
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_resp16=$OPT > gpurun_out/r04l_c4_${OPT}_$I.json 2> gpurun_out/r04l_c4_$I.err \
    || { echo "c4 failed"; tail -20 gpurun_out/r04l_c4_$I.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04l_c4_${OPT}_$I.json'));c=j['config'];print('r16=$OPT', {k:(round(c[k],3) if isinstance(c[k],float) else c[k]) for k in c if k.startswith('gmm_resp') or k.startswith('gmm_em')})"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_tierc.py -m gpu -v -s -k "bench_launch" \
  --timeout 250 --timeout-method thread > gpurun_out/r04l_tierc.log 2>&1
echo "tierc rc=$?"; grep -E "bench launch|passed|failed" gpurun_out/r04l_tierc.log | tail -3
for HP in 0 5e-6; do for LR in 0.1 0.2; do
  timeout -k 10 200 python bench_aux.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline \
    --lr $LR --hot-p $HP > gpurun_out/r04l_c2_${HP}_$LR.json 2> gpurun_out/r04l_c2.err \
    || { echo "c2 failed"; tail -5 gpurun_out/r04l_c2.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04l_c2_${HP}_$LR.json'));print('c2 hot_p=$HP lr=$LR', round(j['roofline']['avg_kernel_ms'],4), 'ms hot rows', j['config']['hot_rows'])"
done; done
