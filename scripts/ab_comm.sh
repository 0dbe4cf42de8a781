set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_c4.sh > gpurun_out/c4_async.log 2>&1 || { tail -30 gpurun_out/c4_async.log; exit 1; }
grep -o "[0-9]* passed.*" gpurun_out/c4_async.log
for v in "" "--opt community_async=0" "" "--opt community_async=0"; do
  timeout -k 10 200 python bench_aux.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline $v > gpurun_out/ab_c4.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_c4.json'));print('$v', d['ms_per_step'], d['roofline']['frac'])"
done
