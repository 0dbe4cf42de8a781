#!/bin/bash
# Round 3 (driver), third pass: A/B of four forms of the stream kernel's prefetched-copy patch at
# the bench launch; bit-exactness of the candidates; multi-rank tier C with hot_mean combines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ABD=$PWD/nodeembedding-to-communityembedding_amd/csrc/build/ab
B="bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary"
for V in select addpatch reload branch select reload branch addpatch; do
  if [ $V = select ]; then unset COME_LIB_PATH; else export COME_LIB_PATH=$ABD/libcome_$V.so; fi
  timeout -k 10 300 python $B > gpurun_out/r04c_ab_$V.json 2> gpurun_out/r04c_ab_$V.err \
    || { echo "bench $V failed"; tail -20 gpurun_out/r04c_ab_$V.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04c_ab_$V.json'));print('$V', round(j['ms_per_step'],2), round(j['roofline']['avg_kernel_ms'],2))"
done
for V in reload branch; do
  export COME_LIB_PATH=$ABD/libcome_$V.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -q -k "bit_exact" --timeout 120 \
    > gpurun_out/r04c_exact_$V.log 2>&1; echo "$V bit-exact tests rc=$?"; tail -2 gpurun_out/r04c_exact_$V.log
done
unset COME_LIB_PATH
timeout -k 10 600 python -u scripts/tierc_replicas.py --fixture c3_1m --worlds 2,4,8 \
  --periods 131072,32768 --combines hot_mean,hot_mean:1e-6,hot_mean:2e-5 \
  --out gpurun_out/r04c_tierc_replicas_c3_1m.json > gpurun_out/r04c_replicas.log 2>&1 \
  || { echo "replicas failed"; tail -20 gpurun_out/r04c_replicas.log; exit 1; }
grep world gpurun_out/r04c_replicas.log | cut -c1-200 | head -40
