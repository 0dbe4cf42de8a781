#!/bin/bash
# Walker output A/B: direct per-lane row stores (walk_staged=0) vs LDS-staged coalesced segments
# (walk_staged=1, the default), after the walker GPU tests (which check the two are identical).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_walks.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_walks.log 2>&1 || { tail -30 gpurun_out/pytest_walks.log; exit 1; }
tail -3 gpurun_out/pytest_walks.log
for opt in ${OPTS:-0 1 0 1}; do
  timeout -k 10 300 python bench_aux.py --workload walks --steps 20 --warmup 3 --no-cpu-baseline \
    --opt walk_staged=$opt > gpurun_out/ab_walks_$opt.json 2> gpurun_out/ab_walks_$opt.err \
    || { tail -20 gpurun_out/ab_walks_$opt.err; exit 1; }
  echo "walk_staged=$opt $(python -c "import json,sys; r=json.load(open(sys.argv[1])); print(r['ms_per_step'], 'ms', r['value'], r['roofline']['frac'])" gpurun_out/ab_walks_$opt.json)"
done
