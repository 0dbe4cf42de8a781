set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/diag_c3.py --repeat 5 --variants stream,direct > gpurun_out/r02ad_diag.log 2>&1 || exit 1
