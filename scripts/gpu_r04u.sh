#!/bin/bash
# Round 3 (driver): E-step variant bits of k_gmm_resp16t (gmm_resp16 = 16 + VT: 1 = paired blocks, 8 = one row tile per wavefront,
# 2 = packed-fp32 epilogue, 4 = next component's staging behind the first A reads), C4 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in 1 2; do
for R in 16 18 24 26 28 30 25; do
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_resp16=$R > gpurun_out/r04u_c4_$R.json 2> gpurun_out/r04u_c4.err \
    || { echo "c4 failed"; tail -20 gpurun_out/r04u_c4.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04u_c4_$R.json'));c=j['config'];print('r16=$R', round(c['gmm_resp_ms'],3), round(c['gmm_resp_tflops_executed'],1))"
done
done
exit 0
