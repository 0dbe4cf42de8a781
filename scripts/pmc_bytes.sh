#!/bin/bash
# Exact fabric read bytes by request size (TCC_EA0_RDREQ_{32B,64B,128B}) and write requests, for a
# command given after --, one rocprofv3 pass per counter group (TCC holds 4 counters per pass).
#   OUT=gpurun_out/x bash scripts/pmc_bytes.sh -- python3 bench.py --steps 3 --warmup 1
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="${OUT:-$ROOT/gpurun_out/pmc_bytes}"
shift  # the --
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for G in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  timeout -s KILL 300 rocprofv3 --pmc $G --output-format csv -d "$OUT/pass$i" -o run -- "$@" > "$OUT/pass$i.out" 2> "$OUT/pass$i.err" || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo done
