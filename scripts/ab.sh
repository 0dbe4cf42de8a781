#!/bin/bash
# A/B of launch variants on one box: the variants run interleaved ROUNDS times (box drift hits
# them alike) and each run's average kernel time is printed.
#   bash scripts/ab.sh TAG "python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary" \
#        ROUNDS "name:extra args" ["name:extra args" ...]
# Variants differ by arguments (e.g. --opt o1_chunk=0) and/or by an alternative build given first
# as "name:COME_LIB_PATH=path [args]" (scripts/build_ab.sh); results in gpurun_out/TAG_ab.txt.  AB_KEYS="k1 k2": also
# print these fields of the JSON line's config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; BASE=$2; ROUNDS=$3; shift 3
OUT=gpurun_out/${TAG}_ab.txt
: > "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for V in "$@"; do
    N=${V%%:*}; A=${V#*:}; ENVV=""
    case "$A" in COME_LIB_PATH=*) ENVV="${A%% *}"; [ "$ENVV" = "$A" ] && A="" || A="${A#* }";; esac
    env $ENVV timeout -k 10 ${AB_SECS:-300} $BASE $A > gpurun_out/${TAG}_$N.json 2> gpurun_out/${TAG}_$N.err \
      || { echo "variant $N failed"; tail -5 gpurun_out/${TAG}_$N.err; exit 1; }
    python3 -c "import json,sys,os; j=json.load(open(sys.argv[1])); r=j.get('roofline') or {}; c=j.get('config') or {}; print(sys.argv[2], sys.argv[3], round(r.get('avg_kernel_ms', j['ms_per_step']), 4), round(r.get('frac', 0), 4), *[(k, c.get(k)) for k in os.environ.get('AB_KEYS', '').split()])" \
      gpurun_out/${TAG}_$N.json "$r" "$N" | tee -a "$OUT"
  done
done
