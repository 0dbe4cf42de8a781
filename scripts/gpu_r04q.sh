#!/bin/bash
# Round 3 (driver): O1 with the input row held over runs of edges (k_sgns_o1_runs, o1_chunk):
# bit-exactness, tier C in the reference's edge order, and C2 timing vs the per-edge kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tierc.py -m gpu -v -s \
  -k "o1" --timeout 300 --timeout-method thread > gpurun_out/r04q_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|G.edges|reference :26" gpurun_out/r04q_pytest.log | tail -10
[ $PYTEST_RC -eq 0 ] || [ $PYTEST_RC -eq 1 ] || exit $PYTEST_RC
for CH in 0 -1 16 0 -1; do
  timeout -k 10 200 python bench_aux.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline \
    --opt o1_chunk=$CH > gpurun_out/r04q_c2_$CH.json 2> gpurun_out/r04q_c2.err \
    || { echo "c2 failed"; tail -5 gpurun_out/r04q_c2.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04q_c2_$CH.json'));print('c2 chunk=$CH', round(j['roofline']['avg_kernel_ms'],4), 'ms', round(j['roofline']['frac'],3))"
done
exit $PYTEST_RC
