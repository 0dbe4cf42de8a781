#!/bin/bash
# Round 3 (driver), fourth pass: the adopted stream kernel (exact cold-row patch, branch form):
# deterministic + C3 tier-C tests, bench line; multi-rank tier C with the hot_mean combines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py -q \
  --timeout 240 --timeout-method thread > gpurun_out/r04d_pytest.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/r04d_pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary \
  > gpurun_out/r04d_bench.json 2> gpurun_out/r04d_bench.err || { echo bench failed; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/r04d_bench.json'));print(j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline']['frac_skip_adjusted'])"
timeout -k 10 700 python -u scripts/tierc_replicas.py --fixture c3_1m --worlds 2,4,8 \
  --periods 131072,32768 --combines hot_mean,hot_mean:1e-6,hot_mean:2e-5 \
  --out gpurun_out/r04d_tierc_replicas_c3_1m.json > gpurun_out/r04d_replicas.log 2>&1 \
  || { echo "replicas failed"; tail -20 gpurun_out/r04d_replicas.log; exit 1; }
grep world gpurun_out/r04d_replicas.log | cut -c1-200 | head -40
