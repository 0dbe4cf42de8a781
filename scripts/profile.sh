#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel: kernel trace + stats, then HBM traffic
# counters in separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r01}
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-secondary ${BENCH_ARGS}"
fatal() { [ "$1" -ne 0 ] && { echo "fatal rc=$1 in $2"; exit "$1"; }; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
fatal $? trace
for C in FETCH_SIZE WRITE_SIZE ${EXTRA_PMC}; do
  timeout -k 10 400 rocprofv3 --pmc ${C//,/ } --output-format csv -d "$OUT/pmc_$C" -o run -- python3 $BENCH > "$OUT/pmc_${C}_bench.json" 2> "$OUT/pmc_${C}_bench.err"
  fatal $? pmc_$C
done
find "$OUT" -name "*.csv" | head -20
exit 0
