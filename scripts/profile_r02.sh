# r02 round evidence for the bench's dominant kernel: kernel trace + stats and FETCH/WRITE_SIZE
# passes (scripts/profile.sh), then exact request-size byte counts (scripts/pmc_bytes.sh).
set -o pipefail
TAG=${TAG:-r02b} STEPS=5 bash scripts/profile.sh > gpurun_out/${TAG:-r02b}_profile.log 2>&1 || exit 1
OUT=$PWD/gpurun_out/pmcb_${TAG:-r02b} bash scripts/pmc_bytes.sh -- python3 $PWD/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/${TAG:-r02b}_pmcb.log 2>&1
