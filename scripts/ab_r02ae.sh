set -o pipefail
mkdir -p gpurun_out
for NV in "200000 20000" "300000 30000" "500000 50000"; do
  set -- $NV
  echo "== nodes $1 walks $2" >> gpurun_out/r02ae_diag.log
  timeout -k 10 300 python -u scripts/diag_tierc.py --no-oracle --nodes $1 --walks $2 --repeat 6 --hot-p 5e-6 --variants hot_p5e-6,direct_hot_p5e-6 >> gpurun_out/r02ae_diag.log 2>&1 || exit 1
done
