#!/bin/bash
# Round 3 (driver), the current tree end to end: the whole GPU suite, smoke, the driver's default
# bench line, rocprofv3 kernel trace + HBM PMC passes of the default launch (profiles/traffic.json),
# and a world-2 rehearsal of the trainers' distributed path (gloo, both ranks on cuda:0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -s \
  > gpurun_out/r04p_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed" gpurun_out/r04p_pytest.log | tail -8
[ $PYTEST_RC -eq 0 ] || [ $PYTEST_RC -eq 1 ] || exit $PYTEST_RC
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04p_smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/r04p_smoke.log; exit 1; }
tail -1 gpurun_out/r04p_smoke.log
START=$(date +%s)
timeout -k 10 500 python bench.py > gpurun_out/r04p_bench.json 2> gpurun_out/r04p_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/r04p_bench.err; exit 1; }
echo "default bench wall $(( $(date +%s) - START )) s"
python -c "import json;j=json.load(open('gpurun_out/r04p_bench.json'));r=j['roofline'];print(j['value'], j['ms_per_step'], r['frac'], r['frac_skip_adjusted'], r['traffic']); print({k:(v if isinstance(v,str) else {kk:vv for kk,vv in v.items() if kk in ('value','ms_per_step','roofline_frac','gmm_resp_ms','gmm_scatter_ms','gmm_em_iteration_ms')}) for k,v in j['secondary'].items()}); print(j['cpu_baseline']['value'], j['cpu_baseline']['cores'])"
TAG=r04p STEPS=5 bash scripts/profile.sh || exit 1
cd "$ROOT" && python scripts/summarize_profile.py gpurun_out/prof_r04p r04p > gpurun_out/r04p_summary.json \
  && grep -E "rocprof_avg|bench_event|actual_hbm|hbm_bytes" gpurun_out/r04p_summary.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
  --dist-backend gloo --all-ranks-device0 --no-cpu-baseline > gpurun_out/r04p_n2.json \
  2> gpurun_out/r04p_n2.err || { echo "n2 rehearsal failed"; tail -30 gpurun_out/r04p_n2.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/r04p_n2.json'));print('n2', j['value'], j['ms_per_step'], j['config']['parallelism'], j['config']['exchanges_per_step'], j['config']['exchange_combine'])"
exit $PYTEST_RC
