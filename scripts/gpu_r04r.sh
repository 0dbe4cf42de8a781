#!/bin/bash
# Round 3 (driver): o1_chunk = -1 as the default -- the full GPU suite, then C2 at the default
# and at the per-edge kernel for the A/B record.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r04r_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|G.edges|reference :26" gpurun_out/r04r_pytest.log | tail -10
[ $PYTEST_RC -eq 0 ] || [ $PYTEST_RC -eq 1 ] || exit $PYTEST_RC
for CH in -1 0 -1 0; do
  timeout -k 10 200 python bench_aux.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline \
    --opt o1_chunk=$CH > gpurun_out/r04r_c2_$CH.json 2> gpurun_out/r04r_c2.err \
    || { echo "c2 failed"; tail -5 gpurun_out/r04r_c2.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04r_c2_$CH.json'));print('c2 chunk=$CH', round(j['roofline']['avg_kernel_ms'],4), 'ms', round(j['roofline']['frac'],3))"
done
exit $PYTEST_RC
