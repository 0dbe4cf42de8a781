#!/bin/bash
# Round-end evidence in one gpurun call: GPU tests + smoke + bench (scripts/gpu_check.sh), then the
# secondary rows' bench lines (C2 O1, C4 community/GMM, walker).  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
for W in c2 c4 walks; do
  timeout -k 10 300 python bench_aux.py --workload $W --steps 20 --warmup 3 > gpurun_out/aux_$W.json \
    2> gpurun_out/aux_$W.err || { echo "bench_aux $W failed"; tail -20 gpurun_out/aux_$W.err; exit 1; }
  cat gpurun_out/aux_$W.json
done
