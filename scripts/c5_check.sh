#!/bin/bash
# C5 (one GPU's shard): write-back A/B, then the bench.py line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_o2.py --nodes 10000000 --dim 256 --negative 10 --rounds 3 \
  --variants default o2_plain_writeback=1 o2_pair_atomics=1 > gpurun_out/ab_c5_wb.txt \
  2> gpurun_out/ab_c5_wb.err || { tail -20 gpurun_out/ab_c5_wb.err; exit 1; }
cat gpurun_out/ab_c5_wb.txt
timeout -k 10 600 python -u bench.py --nodes 10000000 --dim 256 --negative 10 --steps 5 --warmup 1 \
  --no-cpu-baseline > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -20 gpurun_out/c5.err; exit 1; }
cat gpurun_out/c5.json
