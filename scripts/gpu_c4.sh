#!/bin/bash
# One gpurun call for the C4 rows: GPU GMM / community tests, the 1-GPU C4 bench, and a 2-rank
# rehearsal of the row-sharded C4 path on one MI355X (gloo, both ranks on cuda:0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gmm.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "gmm or community or resp" > gpurun_out/c4_pytest.log 2>&1 \
  || { tail -30 gpurun_out/c4_pytest.log; exit 1; }
tail -3 gpurun_out/c4_pytest.log
timeout -k 10 300 python bench_aux.py --workload c4 --steps 10 --warmup 2 \
  > gpurun_out/c4_n1.json 2> gpurun_out/c4_n1.err || { tail -20 gpurun_out/c4_n1.err; exit 1; }
cat gpurun_out/c4_n1.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench_aux.py --workload c4 --steps 5 --warmup 1 \
  --dist-backend gloo --all-ranks-device0 > gpurun_out/c4_n2_rehearsal.json \
  2> gpurun_out/c4_n2_rehearsal.err || { tail -20 gpurun_out/c4_n2_rehearsal.err; exit 1; }
cat gpurun_out/c4_n2_rehearsal.json
