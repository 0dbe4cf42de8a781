#!/bin/bash
# r03: per-launch tail of the streaming O2 kernel -- C3 kernel time per 1e8 pairs at batch sizes
# of 65,536 / 131,072 / 262,144 walks per launch (a fixed tail shows up as a per-launch constant).
set -o pipefail
mkdir -p gpurun_out
for B in 65536 131072 262144; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary --walks-per-step $B > gpurun_out/r03i_b$B.json 2> gpurun_out/r03i_b$B.err || { tail -3 gpurun_out/r03i_b$B.err; exit 1; }
  python -c "import json; j=json.load(open('gpurun_out/r03i_b$B.json')); p=j['config']['pairs_per_step_per_gpu']; k=j['roofline']['avg_kernel_ms']; print('walks $B kernel_ms %.2f pairs %.4g ms_per_1e8 %.2f step_ms %.2f' % (k, p, k/p*1e8, j['ms_per_step']))"
done
