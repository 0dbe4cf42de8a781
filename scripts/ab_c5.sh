#!/bin/bash
# C5 (one GPU's shard: 10M nodes, d=256, n=10) O2 grid A/B, then the C2 bench at the new O1 default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/ab_o2.py --nodes 10000000 --dim 256 --negative 10 --rounds 3 \
  --variants default resident_cap=1 o2_blocks_per_cu=5 o2_blocks_per_cu=4 \
  o2_waves_per_block=1 o2_waves_per_block=1,o2_blocks_per_cu=12 \
  o2_waves_per_block=1,o2_blocks_per_cu=10 > gpurun_out/ab_c5.txt 2> gpurun_out/ab_c5.err \
  || { tail -20 gpurun_out/ab_c5.err; exit 1; }
cat gpurun_out/ab_c5.txt
timeout -k 10 200 python bench_aux.py --workload c2 --steps 50 --warmup 5 > gpurun_out/c2.json \
  2> gpurun_out/c2.err || { tail -20 gpurun_out/c2.err; exit 1; }
cat gpurun_out/c2.json
