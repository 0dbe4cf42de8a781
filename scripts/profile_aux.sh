#!/bin/bash
# rocprofv3 kernel traces of the bench's secondary rows (bench_aux.py c2 / c4 / walks, the same
# commands bench.py runs, without their CPU baselines), then FETCH_SIZE / WRITE_SIZE passes of the
# C2 O1 kernel.  Each run under its own time limit; the first failure ends the script.
#   TAG=r06_aux bash scripts/profile_aux.sh
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-aux}
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for WL in c2 c4 walks; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$WL" -o run -- \
    python3 "$ROOT/bench_aux.py" --workload $WL --steps 10 --warmup 2 --no-cpu-baseline \
    > "$OUT/${WL}.json" 2> "$OUT/${WL}.err" || { echo "trace $WL failed"; exit 1; }
  echo "trace $WL done"
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/c2_$C" -o run -- \
    python3 "$ROOT/bench_aux.py" --workload c2 --steps 10 --warmup 2 --no-cpu-baseline \
    > "$OUT/c2_${C}.json" 2> "$OUT/c2_${C}.err" || { echo "pmc $C failed"; exit 1; }
  echo "pmc $C done"
done
exit 0
