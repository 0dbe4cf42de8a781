#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a short run; each pass has its own time
# limit.  Usage: TAG=x [CMD="bench_aux.py --workload c2 ..."] [KERNEL=sgns_o1] \
#   bash scripts/pmc.sh "SQ_WAVE_CYCLES SQ_WAIT_ANY" "TCC_HIT_sum TCC_MISS_sum"
# CMD (default: a short bench.py run) is a python script + arguments relative to the repo root;
# per-launch sums are reported for kernels whose name contains KERNEL (default sgns_o2).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-pmc}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/${CMD:-bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-secondary ${BENCH_ARGS}}"
export KERNEL=${KERNEL:-sgns_o2}
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o run -- python3 $BENCH > "$OUT/p${i}.json" 2> "$OUT/p${i}.err"
  rc=$?; [ $rc -ne 0 ] && { echo "pass $i ($C) rc=$rc"; tail -3 "$OUT/p${i}.err"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if os.environ["KERNEL"] not in r.get("Kernel_Name", ""):
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r.get("Dispatch_Id", ""))
for k in sorted(agg):
    print("%-28s per-launch %.4g  (launches=%d)" % (k, agg[k] / max(1, len(disp[k])),
                                                   len(disp[k])))
PY
