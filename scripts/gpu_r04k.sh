#!/bin/bash
# Round 3 (driver): the device chung_lu rebuilt from 1-D ops (torch's large 2-D row gathers are
# wrong on this ROCm build): gather probe, device-vs-host C5 inputs, then the C5 tier-C test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/bisect_torch_gather.py > gpurun_out/r04k_gather.log 2>&1
echo "gather probe rc=$?"; grep -v amdgpu.ids gpurun_out/r04k_gather.log | tail -4
timeout -k 10 400 python -u scripts/check_c5_inputs.py > gpurun_out/r04k_check.log 2>&1 \
  || { echo "check failed"; tail -20 gpurun_out/r04k_check.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04k_check.log | tail -8
timeout -k 10 600 python -u -m pytest tests/test_gpu_tierc.py -m gpu -v -s -k "c5" --timeout 500 \
  --timeout-method thread > gpurun_out/r04k_pytest.log 2>&1
rc=$?
grep -E "V=|passed|failed|Error" gpurun_out/r04k_pytest.log | tail -8
exit $rc
