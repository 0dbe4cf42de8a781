# r02u: GMM tests + C4 bench (2-component scatter), then C3 plain vs packed negative table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gmm.py -q -x --timeout 300 --timeout-method thread > gpurun_out/r02u_gmm.log 2>&1 || exit 1
timeout -k 10 200 python bench_aux.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02u_c4.json 2> gpurun_out/r02u_c4.err || exit 1
for V in "" "--packed-table" "" "--packed-table"; do
  echo "== [$V]" >> gpurun_out/r02u_c3.log
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $V >> gpurun_out/r02u_c3.log 2>/dev/null || exit 1
done
