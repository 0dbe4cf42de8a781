#!/bin/bash
# Round 3 (driver), ninth pass: the whole GPU suite on the current tree (C5 tier C against the new
# 10M-node fixture, the CPU-twin test, k_gmm_resp16 default) and smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s \
  > gpurun_out/r04i_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|V=10000000|held-out" gpurun_out/r04i_pytest.log | tail -15
[ $PYTEST_RC -eq 0 ] || [ $PYTEST_RC -eq 1 ] || exit $PYTEST_RC
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04i_smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/r04i_smoke.log; exit 1; }
tail -1 gpurun_out/r04i_smoke.log
exit $PYTEST_RC
