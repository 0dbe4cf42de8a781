#!/bin/bash
# PMC passes over a short C4 run (bench_aux.py --workload c4): one rocprofv3 run per counter group.
#   [C4_ARGS="--opt community_async=3"] [TAG=name] bash scripts/pmc_c4.sh "CTR1 CTR2" "CTR3" ...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_c4${TAG:+_$TAG}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RUN="$ROOT/bench_aux.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline ${C4_ARGS:-}"
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o run -- python3 $RUN > "$OUT/p${i}.json" 2> "$OUT/p${i}.err"
  rc=$?; [ $rc -ne 0 ] && { echo "pass $i ($C) rc=$rc"; tail -3 "$OUT/p${i}.err"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r.get("Kernel_Name", "")
        for tag in ("k_community_async", "k_community16", "k_community_bf3", "k_gmm_resp16t",
                    "k_gmm_resp_mfma", "k_gmm_cov_async", "k_gmm_cov16", "k_gmm_cov_bf3",
                    "k_gmm_resp_bf3", "k_community_b16", "k_gmm_resp_b16", "k_gmm_cov_fb3"):
            if tag in kn:
                key = (tag, r["Counter_Name"])
                agg[key] += float(r["Counter_Value"])
                disp[key].add(r.get("Dispatch_Id", ""))
for k in sorted(agg):
    print("%-18s %-30s per-launch %.4g  (launches=%d)" % (k[0], k[1], agg[k] / max(1, len(disp[k])),
                                                        len(disp[k])))
PY
