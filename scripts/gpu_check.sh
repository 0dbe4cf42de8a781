#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench.  Every GPU step has its own time limit; a
# timeout / signal / crash (rc >= 124) ends the script, a plain test failure does not.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
fatal() { [ "$1" -ge 124 ] && { echo "fatal rc=$1 in $2"; exit "$1"; }; }
timeout -k 10 600 python -m pytest tests -m gpu -q -rs ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; cat gpurun_out/smoke.log | tail -5; fatal $rc smoke
timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json; fatal $rc bench
exit 0
