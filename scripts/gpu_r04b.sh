#!/bin/bash
# Round 3 (driver), second pass: (1) A/B of the stream kernel's prefetched-copy patch (exact
# replacement for cold rows vs round 2's additive patch: libcome_addpatch.so) at the bench launch,
# A-B-A; (2) multi-rank tier C with the averaging combine rules; (3) C5 tier C vs waves in flight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB=nodeembedding-to-communityembedding_amd/csrc/build/ab/libcome_addpatch.so
B="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary"
for V in new old new; do
  if [ $V = old ]; then export COME_LIB_PATH=$PWD/$AB; else unset COME_LIB_PATH; fi
  timeout -k 10 300 python $B > gpurun_out/r04b_ab_$V.json 2> gpurun_out/r04b_ab_$V.err \
    || { echo "bench $V failed"; tail -20 gpurun_out/r04b_ab_$V.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04b_ab_$V.json'));print('$V', j['ms_per_step'], j['roofline']['avg_kernel_ms'])"
done
unset COME_LIB_PATH
timeout -k 10 600 python -u scripts/tierc_replicas.py --fixture c3_1m --worlds 2,4,8 \
  --periods 131072,32768,8192 --combines touched_mean,mean \
  --out gpurun_out/r04b_tierc_replicas_c3_1m.json > gpurun_out/r04b_replicas.log 2>&1 \
  || { echo "replicas failed"; tail -20 gpurun_out/r04b_replicas.log; exit 1; }
grep world gpurun_out/r04b_replicas.log | head -40
timeout -k 10 400 python -u scripts/tierc_c5_waves.py --out gpurun_out/r04b_c5_waves.json \
  > gpurun_out/r04b_c5_waves.log 2>&1 || { echo "c5 waves failed"; tail -20 gpurun_out/r04b_c5_waves.log; exit 1; }
cat gpurun_out/r04b_c5_waves.log | grep max_waves
