#!/bin/bash
# Round 3 (driver): (1) C5 one-GPU shard with the stream kernel at 2 (default, 181 VGPRs) vs 3 waves
# per SIMD (alt build, 168 VGPRs + 96 B spill); (2) the multi-rank exchange at sync periods of up to
# 524,288 walks per rank against the 4,194,304-walk sequential fixture (C3_4M).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C5="--nodes 10000000 --dim 256 --negative 10 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary"
timeout -k 10 400 python bench.py $C5 > gpurun_out/r04n_c5_w2.json 2> gpurun_out/r04n_c5_w2.err \
  || { echo "c5 w2 failed"; tail -5 gpurun_out/r04n_c5_w2.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/r04n_c5_w2.json'));r=j['roofline'];print('c5 w2', j['value'], r['avg_kernel_ms'], r['frac'], r['frac_skip_adjusted'])"
COME_LIB_PATH=$(pwd)/nodeembedding-to-communityembedding_amd/alt/libcome_w3.so timeout -k 10 400 \
  python bench.py $C5 > gpurun_out/r04n_c5_w3.json 2> gpurun_out/r04n_c5_w3.err \
  || { echo "c5 w3 failed"; tail -5 gpurun_out/r04n_c5_w3.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/r04n_c5_w3.json'));r=j['roofline'];print('c5 w3', j['value'], r['avg_kernel_ms'], r['frac'], r['frac_skip_adjusted'])"
timeout -k 10 900 python -u scripts/tierc_replicas.py --fixture c3_4m --worlds 1,2,4,8 \
  --periods 524288,262144,131072 --out gpurun_out/r04n_tierc_replicas_c3_4m.json \
  > gpurun_out/r04n_replicas.log 2>&1 || { echo "replicas failed"; tail -20 gpurun_out/r04n_replicas.log; exit 1; }
grep world gpurun_out/r04n_replicas.log | cut -c1-220
