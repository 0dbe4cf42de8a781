#!/bin/bash
# Round 3 (driver): rocprofv3 kernel-trace stats of the C4 row on the current defaults
# (k_community16, k_gmm_resp16t one-tile form, k_gmm_cov16), csv output.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_r04za" -o run -- \
  python3 "$ROOT/bench_aux.py" --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
  > "$ROOT/gpurun_out/r04za_c4.json" 2> "$ROOT/gpurun_out/r04za_c4.err" || { echo "trace failed"; tail -5 "$ROOT/gpurun_out/r04za_c4.err"; exit 1; }
f=$(find "$ROOT/gpurun_out/prof_r04za" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] || { echo "no stats file"; find "$ROOT/gpurun_out/prof_r04za" | head; exit 1; }
cp "$f" "$ROOT/gpurun_out/r04za_kernel_stats.csv"
grep -E "community16|resp16|cov16|cov_reduce|Name" "$f" | cut -c1-220
python3 -c "import json;j=json.load(open('$ROOT/gpurun_out/r04za_c4.json'));c=j['config'];print(j['ms_per_step'], c['gmm_resp_ms'], c['gmm_scatter_ms'], c['gmm_em_iteration_ms'])"
