#!/bin/bash
# Round 3 (driver): E-step epilogue A/B, then evidence for the C4 defaults (k_community16, k_gmm_resp16t one-tile form,
# k_gmm_cov16): rocprofv3 kernel-trace stats of the C4 row, and one SQ PMC pass (MFMA busy).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gmm.py -m gpu -v -k "estep" \
  --timeout 200 --timeout-method thread > gpurun_out/r04z_pytest.log 2>&1
PYTEST_RC=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/r04z_pytest.log | tail -12
[ $PYTEST_RC -eq 0 ] || exit $PYTEST_RC
timeout -k 10 120 python - <<'PY' || exit 1
import numpy as np, torch
from come_amd import _lib, gmm
rng = np.random.RandomState(5)
for V, K, d in ((4097, 50, 128), (3001, 7, 64)):
    X = rng.standard_normal((V, d)).astype(np.float32)
    P = np.stack([np.triu(rng.standard_normal((d, d)) / np.sqrt(d)) + 2 * np.eye(d) for _ in range(K)])
    mp = np.einsum("kd,kde->ke", rng.standard_normal((K, d)) * 0.3, P)
    ln = np.log(rng.dirichlet(np.ones(K)))
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float32), device="cuda")
    out = {}
    for r in (2, 20, 21, 22):
        _lib.set_option("gmm_resp16", r)
        resp, lse = gmm.estep(t(X), t(P), t(mp), t(ln))
        out[r] = resp.cpu().numpy(), lse.cpu().numpy()
    _lib.set_option("gmm_resp16", 2)
    for r in (20, 21, 22):
        dr = np.abs(out[r][0] - out[2][0]).max(); dl = np.abs(out[r][1] - out[2][1]).max()
        print("variant", r, "d", d, "max |resp diff|", dr, "max |lse diff|", dl)
        assert dr < 1e-4 and dl < 1e-3
PY
# E-step epilogue variants: 20 = log-sum-exp after the loop, 21 = accumulators from -mu P, 22 = both
for P in 1 2; do
for R in 2 20 21 22; do
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
    --opt gmm_resp16=$R > gpurun_out/r04z_ab_$R.json 2> gpurun_out/r04z_ab.err \
    || { echo "c4 failed"; tail -20 gpurun_out/r04z_ab.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/r04z_ab_$R.json'));c=j['config'];print('r16=$R', round(c['gmm_resp_ms'],3), round(c['gmm_resp_tflops_executed'],1))"
done
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_r04z" -o run -- \
  python3 "$ROOT/bench_aux.py" --workload c4 --steps 10 --warmup 2 --no-cpu-baseline \
  > "$ROOT/gpurun_out/r04z_c4.json" 2> "$ROOT/gpurun_out/r04z_c4.err" || { echo "trace failed"; tail -5 "$ROOT/gpurun_out/r04z_c4.err"; exit 1; }
f=$(find "$ROOT/gpurun_out/prof_r04z" -name "*kernel_stats.csv" | head -1)
cp "$f" "$ROOT/gpurun_out/r04z_kernel_stats.csv"
grep -E "community16|resp16|cov16|cov_reduce|Name" "$f" | cut -c1-200
OUT="$ROOT/gpurun_out/pmc_r04z"
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d "$OUT/p1" -o run -- \
  python3 "$ROOT/bench_aux.py" --workload c4 --steps 3 --warmup 1 --no-cpu-baseline \
  > "$OUT/p1.json" 2> "$OUT/p1.err"
rc=$?; [ $rc -ne 0 ] && { echo "pmc rc=$rc"; tail -3 "$OUT/p1.err"; exit $rc; }
cd "$ROOT"
python3 - "$OUT" <<'PY' | tee gpurun_out/r04z_pmc.txt
import csv, glob, sys, collections
out = sys.argv[1]
for kn in ("k_community16", "k_gmm_resp16t", "k_gmm_cov16"):
    agg = collections.defaultdict(float); disp = collections.defaultdict(set)
    for f in glob.glob(out + "/p1/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kn in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r.get("Dispatch_Id", ""))
    per = {k: v / max(1, len(disp[k])) for k, v in agg.items()}
    busy = per.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / max(1.0, per.get("GRBM_GUI_ACTIVE", 1) / 8)
    print(kn, "launches", max([len(x) for x in disp.values()] or [0]), {k: "%.4g" % v for k, v in sorted(per.items())}, "mfma_busy_frac %.3f" % busy)
PY
exit 0
