#!/bin/bash
# Round 3 (driver): the stream kernel's cold-row patch as the row update's own fma (one code path
# for hot and cold copies: C5's kernel back to 149 VGPRs / 3 waves per SIMD) vs the branch form
# (alt build, 181 VGPRs / 2 waves): exactness tests, tier C at C3 / C5, and C3 + C5 timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py tests/test_gpu_tierc.py \
  -m gpu -v -s --timeout 400 --timeout-method thread -k "not multi_rank" > gpurun_out/r04o_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|V=|bench launch|held-out" gpurun_out/r04o_pytest.log | tail -14
[ $PYTEST_RC -eq 0 ] || exit $PYTEST_RC
ALT=$(pwd)/nodeembedding-to-communityembedding_amd/alt/libcome_branch.so
C3="--steps 6 --warmup 2 --no-cpu-baseline --no-secondary"
C5="--nodes 10000000 --dim 256 --negative 10 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary"
for V in fma branch fma branch; do
  if [ $V = fma ]; then unset COME_LIB_PATH; else export COME_LIB_PATH=$ALT; fi
  timeout -k 10 300 python bench.py $C3 > gpurun_out/r04o_c3_$V.json 2> gpurun_out/r04o_c3_$V.err \
    || { echo "c3 $V failed"; tail -5 gpurun_out/r04o_c3_$V.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04o_c3_$V.json'));r=j['roofline'];print('c3 $V', round(r['avg_kernel_ms'],2), round(r['frac'],4), round(r['frac_skip_adjusted'],4))"
done
for V in fma branch; do
  if [ $V = fma ]; then unset COME_LIB_PATH; else export COME_LIB_PATH=$ALT; fi
  timeout -k 10 400 python bench.py $C5 > gpurun_out/r04o_c5_$V.json 2> gpurun_out/r04o_c5_$V.err \
    || { echo "c5 $V failed"; tail -5 gpurun_out/r04o_c5_$V.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04o_c5_$V.json'));r=j['roofline'];print('c5 $V', j['value'], round(r['avg_kernel_ms'],1), round(r['frac'],4), round(r['frac_skip_adjusted'],4))"
done
