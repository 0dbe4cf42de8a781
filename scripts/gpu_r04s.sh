#!/bin/bash
# Round 3 (driver): persistent split-component E-step k_gmm_resp16p (gmm_resp16 = 3) -- GMM tests,
# then C4 A/B against k_gmm_resp16t (= 2), alternating, and a kernel trace of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gmm.py -m gpu -v -k "estep" \
  --timeout 200 --timeout-method thread > gpurun_out/r04s_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r04s_pytest.log | tail -12
[ $PYTEST_RC -eq 0 ] || exit $PYTEST_RC
for R in 2 3 2 3; do
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_resp16=$R > gpurun_out/r04s_c4_$R.json 2> gpurun_out/r04s_c4.err \
    || { echo "c4 failed"; tail -20 gpurun_out/r04s_c4.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04s_c4_$R.json'));c=j['config'];print('r16=$R', {k:(round(c[k],3) if isinstance(c[k],float) else c[k]) for k in c if k.startswith('gmm_resp') or k=='gmm_em_iteration_ms'})"
done
ROOT=$(pwd)
cd /tmp
for R in 2 3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_r04s_$R" -o run -- \
    python3 "$ROOT/bench_aux.py" --workload c4 --steps 5 --warmup 1 --no-cpu-baseline \
    --opt gmm_resp16=$R > "$ROOT/gpurun_out/r04s_prof_$R.log" 2>&1 || { echo "prof $R failed"; exit 1; }
  f=$(find "$ROOT/gpurun_out/prof_r04s_$R" -name "*kernel_stats.csv" | head -1)
  grep -E "resp16|fix" "$f" | cut -c1-160
done
exit 0
