set -o pipefail
mkdir -p gpurun_out
for v in "" "--opt no_resident_cap=1" "--opt o1_blocks_per_cu=6" "--opt o1_blocks_per_cu=5" "" "--opt no_resident_cap=1" "--opt o1_blocks_per_cu=4"; do
  echo "variant: $v" >> gpurun_out/ab_c2.txt
  timeout -k 10 200 python bench_aux.py --workload c2 --steps 50 --warmup 5 --no-cpu-baseline $v > gpurun_out/ab_one.json 2>>gpurun_out/ab_c2.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_one.json'));print(d['roofline']['avg_kernel_ms'], d['value'], d['roofline']['frac'])" >> gpurun_out/ab_c2.txt
done
cat gpurun_out/ab_c2.txt
