#!/bin/bash
# Round 3 (driver), first GPU pass: the GPU tests (new deterministic stream-kernel tests, C5 and
# multi-rank tier C), smoke, the default bench line, the multi-rank tier-C curve, and a world-2
# gloo rehearsal of the trainers' distributed path with both ranks on cuda:0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
  > gpurun_out/r04a_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed" gpurun_out/r04a_pytest.log | tail -15
[ $PYTEST_RC -eq 0 ] || [ $PYTEST_RC -eq 1 ] || exit $PYTEST_RC   # 1 = test failures: go on
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04a_smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/r04a_smoke.log; exit 1; }
tail -1 gpurun_out/r04a_smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a_bench.json \
  2> gpurun_out/r04a_bench.err || { echo "bench failed"; tail -20 gpurun_out/r04a_bench.err; exit 1; }
cat gpurun_out/r04a_bench.json
timeout -k 10 600 python -u scripts/tierc_replicas.py --fixture c3_1m \
  --out gpurun_out/r04a_tierc_replicas_c3_1m.json > gpurun_out/r04a_replicas.log 2>&1 \
  || { echo "replicas failed"; tail -20 gpurun_out/r04a_replicas.log; exit 1; }
grep world gpurun_out/r04a_replicas.log | head -40
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
  --dist-backend gloo --all-ranks-device0 --no-cpu-baseline --sync-walks 524288 > gpurun_out/r04a_n2.json \
  2> gpurun_out/r04a_n2.err || { echo "n2 rehearsal failed"; tail -30 gpurun_out/r04a_n2.err; exit 1; }
cat gpurun_out/r04a_n2.json
for OPT in 0 1; do
  timeout -k 10 300 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_resp_db=$OPT > gpurun_out/r04a_c4_db$OPT.json 2> gpurun_out/r04a_c4_db$OPT.err \
    || { echo "c4 db=$OPT failed"; tail -20 gpurun_out/r04a_c4_db$OPT.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04a_c4_db$OPT.json'));c=j['config'];print('db=$OPT', {k:c[k] for k in c if k.startswith('gmm')})"
done
exit $PYTEST_RC
