set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/diag_tierc.py --no-oracle --repeat 10 --hot-p 5e-6,1e-9 --variants hot_p5e-6,direct_hot_p5e-6,direct_fresh_atomic,hot_p1e-9,stream_nohot > gpurun_out/r02ac_diag.log 2>&1 || exit 1
