set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "sync or community or subset" > gpurun_out/r02n_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/r02n_pytest.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --measure-sync > gpurun_out/r02n_c3_sync.json 2> gpurun_out/r02n_c3_sync.err || exit 1
timeout -k 10 700 python bench.py --nodes 10000000 --dim 256 --negative 10 --steps 3 --warmup 1 --no-cpu-baseline --measure-sync > gpurun_out/r02n_c5_sync.json 2> gpurun_out/r02n_c5_sync.err
