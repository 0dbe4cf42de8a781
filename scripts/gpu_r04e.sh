#!/bin/bash
# Round 3 (driver), fifth pass, on the tree restored after the session cut: the whole GPU suite,
# smoke, the driver's default bench line, and the rocprofv3 kernel trace + HBM PMC passes of the
# adopted stream kernel (profiles/traffic.json keyed to the default launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04e_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed" gpurun_out/r04e_pytest.log | tail -15
[ $PYTEST_RC -eq 0 ] || [ $PYTEST_RC -eq 1 ] || exit $PYTEST_RC   # 1 = test failures: go on
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04e_smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/r04e_smoke.log; exit 1; }
tail -1 gpurun_out/r04e_smoke.log
START=$(date +%s)
timeout -k 10 500 python bench.py > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/r04e_bench.err; exit 1; }
echo "default bench wall $(( $(date +%s) - START )) s"
cat gpurun_out/r04e_bench.json
TAG=r04e STEPS=5 bash scripts/profile.sh || exit 1
cd "$ROOT" && python scripts/summarize_profile.py gpurun_out/prof_r04e r04e > gpurun_out/r04e_summary.json \
  && grep -E "rocprof_avg|bench_event|actual_hbm|hbm_bytes" gpurun_out/r04e_summary.json
I=0
for OPT in 0 1 2 3 0 2 3; do
  I=$((I+1))
  timeout -k 10 300 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_resp_db=$OPT > gpurun_out/r04e_c4_db${OPT}_$I.json 2> gpurun_out/r04e_c4_db${OPT}_$I.err \
    || { echo "c4 db=$OPT failed"; tail -20 gpurun_out/r04e_c4_db${OPT}_$I.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04e_c4_db${OPT}_$I.json'));c=j['config'];print('db=$OPT', {k:c[k] for k in c if k.startswith('gmm')})"
done
exit $PYTEST_RC
