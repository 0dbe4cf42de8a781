#!/bin/bash
# Round 3 (driver): the tree at the end of the session (final tree) --
# the whole GPU suite, smoke and the driver's default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -s \
  > gpurun_out/r04zb_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed" gpurun_out/r04zb_pytest.log | tail -8
[ $PYTEST_RC -eq 0 ] || [ $PYTEST_RC -eq 1 ] || exit $PYTEST_RC
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04zb_smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/r04zb_smoke.log; exit 1; }
tail -1 gpurun_out/r04zb_smoke.log
START=$(date +%s)
timeout -k 10 500 python bench.py > gpurun_out/r04zb_bench.json 2> gpurun_out/r04zb_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/r04zb_bench.err; exit 1; }
echo "default bench wall $(( $(date +%s) - START )) s"
python -c "import json;j=json.load(open('gpurun_out/r04zb_bench.json'));r=j['roofline'];print(j['value'], j['ms_per_step'], r['frac'], r['frac_skip_adjusted'], r['traffic']); print({k:(v if isinstance(v,str) else {kk:vv for kk,vv in v.items() if kk in ('value','ms_per_step','roofline_frac','gmm_resp_ms','gmm_scatter_ms','gmm_em_iteration_ms')}) for k,v in j['secondary'].items()}); print(j['cpu_baseline']['value'], j['cpu_baseline']['cores'])"
exit $PYTEST_RC
