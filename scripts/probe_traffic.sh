#!/bin/bash
# Calibrate FETCH_SIZE / WRITE_SIZE on known byte counts in the O2 kernel's access patterns
# (scripts/traffic_probe.hip, built in the container), one rocprofv3 pass per counter.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/probe_${TAG:-r02}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P="$ROOT/scripts/traffic_probe"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "$P" > "$OUT/known.json" 2> "$OUT/trace.err" || { echo "trace failed"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o run -- "$P" > /dev/null 2> "$OUT/pmc_$C.err" || { echo "pmc $C failed"; exit 1; }
done
find "$OUT" -name "*.csv"
