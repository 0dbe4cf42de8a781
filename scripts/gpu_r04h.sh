#!/bin/bash
# Round 3 (driver), eighth pass: k_gmm_resp16 as the default E-step -- the GMM / C4 GPU tests, the
# C4 row (default options), and the default bench's secondary rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_gmm.py tests/test_gpu_c4.py tests/test_distributed_c4.py -m gpu -v \
  --timeout 200 --timeout-method thread > gpurun_out/r04h_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r04h_pytest.log | tail -12
[ $PYTEST_RC -eq 0 ] || exit $PYTEST_RC
for I in 1 2; do
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r04h_c4_$I.json 2> gpurun_out/r04h_c4_$I.err \
    || { echo "c4 failed"; tail -20 gpurun_out/r04h_c4_$I.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04h_c4_$I.json'));c=j['config'];print({k:(round(c[k],3) if isinstance(c[k],float) else c[k]) for k in c if k.startswith('gmm')})"
done
for I in 3 4; do
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_resp16=2 > gpurun_out/r04h_c4_rot_$I.json 2> gpurun_out/r04h_c4_rot_$I.err \
    || { echo "c4 rot failed"; tail -20 gpurun_out/r04h_c4_rot_$I.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04h_c4_rot_$I.json'));c=j['config'];print('rot', {k:(round(c[k],3) if isinstance(c[k],float) else c[k]) for k in c if k.startswith('gmm_resp')})"
done
ROOT=$(pwd)
OUT="$ROOT/gpurun_out/pmc_r04h"
mkdir -p "$OUT"
cd /tmp
i=0
for OPT in 1 2; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d "$OUT/p${i}" -o run -- \
    python3 "$ROOT/bench_aux.py" --workload c4 --steps 3 --warmup 1 --no-cpu-baseline \
    --opt gmm_resp16=$OPT > "$OUT/p${i}.json" 2> "$OUT/p${i}.err"
  rc=$?; [ $rc -ne 0 ] && { echo "pmc pass $i rc=$rc"; tail -3 "$OUT/p${i}.err"; exit $rc; }
done
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(out + "/p*/")):
    agg = collections.defaultdict(float); disp = collections.defaultdict(set)
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_gmm_resp16" in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r.get("Dispatch_Id", ""))
    print(d, {k: "%.4g" % (v / max(1, len(disp[k]))) for k, v in sorted(agg.items())})
PY
