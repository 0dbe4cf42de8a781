#!/bin/bash
# Round 3 (driver): why the C5 tier-C inputs built on the device differ from the host-built ones.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/check_c5_inputs.py > gpurun_out/r04j_check.log 2>&1
rc=$?; cat gpurun_out/r04j_check.log | tail -30; exit $rc
