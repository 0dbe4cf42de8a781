#!/bin/bash
# Walker (k_random_walks_staged) memory requests per walk step: L2 -> fabric read requests by size,
# L2 hits / misses, one rocprofv3 pass per counter group, over bench_aux.py --workload walks.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_walks"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RUN="$ROOT/bench_aux.py --workload walks --steps 3 --warmup 1 --no-cpu-baseline"
i=0
for G in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  timeout -s KILL 240 rocprofv3 --pmc $G --output-format csv -d "$OUT/p$i" -o run -- python3 $RUN > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pass $i failed"; tail -3 "$OUT/p$i.err"; exit 1; }
  i=$((i+1))
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
agg = collections.defaultdict(float); disp = collections.defaultdict(set)
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_random_walks" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r["Dispatch_Id"])
j = json.load(open(out + "/p0.json"))
steps = j["value"] * j["ms_per_step"] / 1e3  # walk steps per launch
res = {k: agg[k] / len(disp[k]) for k in agg}
res["walk_steps_per_launch"] = steps
res["read_requests_per_step"] = res.get("TCC_EA0_RDREQ_sum", 0) / steps
res["kernel_ms"] = j["roofline"]["avg_kernel_ms"]
print(json.dumps(res, indent=1))
PY
