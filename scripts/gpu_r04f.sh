#!/bin/bash
# Round 3 (driver), sixth pass: CPU-twin vs GPU sequential test, the E-step variant tests; C2 at
# lr 0.1 vs 0.2 (the C2 row read 1.345 ms in r04e vs 1.20-1.24 ms in round 2 at lr 0.2); SQ counters
# of the E-step kernels (k_gmm_resp_mfma vs k_gmm_resp_db) to locate the idle MFMA cycles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_cpu_twins.py tests/test_gpu_gmm.py -m gpu -v \
  --timeout 200 --timeout-method thread > gpurun_out/r04f_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed" gpurun_out/r04f_pytest.log | tail -8
[ $PYTEST_RC -eq 0 ] || [ $PYTEST_RC -eq 1 ] || exit $PYTEST_RC
for LR in 0.1 0.2 0.1 0.2; do
  timeout -k 10 200 python bench_aux.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline \
    --lr $LR > gpurun_out/r04f_c2_lr$LR.json 2> gpurun_out/r04f_c2_lr$LR.err \
    || { echo "c2 lr=$LR failed"; tail -20 gpurun_out/r04f_c2_lr$LR.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04f_c2_lr$LR.json'));print('c2 lr=$LR', round(j['roofline']['avg_kernel_ms'],4), 'ms', round(j['roofline']['frac'],3))"
done
OUT="$ROOT/gpurun_out/pmc_r04f"
mkdir -p "$OUT"
cd /tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "GRBM_GUI_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAVES"; do
  for OPT in 0 1; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p${i}_db$OPT" -o run -- \
      python3 "$ROOT/bench_aux.py" --workload c4 --steps 3 --warmup 1 --no-cpu-baseline \
      --opt gmm_resp_db=$OPT > "$OUT/p${i}.json" 2> "$OUT/p${i}.err"
    rc=$?; [ $rc -ne 0 ] && { echo "pmc pass $i rc=$rc"; tail -3 "$OUT/p${i}.err"; exit $rc; }
  done
done
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, os
out = sys.argv[1]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r.get("Kernel_Name", "")
        for tag in ("k_community_async", "k_gmm_resp_mfma", "k_gmm_resp_db", "k_gmm_cov_async"):
            if tag in kn:
                key = (tag, r["Counter_Name"])
                agg[key] += float(r["Counter_Value"])
                disp[key].add((f, r.get("Dispatch_Id", "")))
for k in sorted(agg):
    print("%-18s %-28s per-launch %.4g  (launches=%d)" % (k[0], k[1], agg[k] / max(1, len(disp[k])),
                                                        len(disp[k])))
PY
exit $PYTEST_RC
