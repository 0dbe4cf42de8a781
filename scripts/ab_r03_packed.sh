#!/bin/bash
# r03: product default = packed negative table + non-temporal negative-row loads (stream kernel).
# O2 parity tests, tier C at C3 with the packed table, C3 bench packed vs plain, C2 packed vs plain.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03f}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tierc.py -x -q \
  --timeout 300 --timeout-method thread -k "o2 or packed or benchmarked" > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${T}_pytest.log; [ $rc -ne 0 ] && exit $rc
for V in "packed:" "plain:--plain-table" "packed2:"; do
  N=${V%%:*}; A=${V#*:}
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary $A > gpurun_out/${T}_c3_$N.json 2> gpurun_out/${T}_c3_$N.err || exit 1
  python -c "import json; j=json.load(open('gpurun_out/${T}_c3_$N.json')); print('c3 $N', round(j['roofline']['avg_kernel_ms'],2), j['config']['negative_table'])"
done
for V in "plain:" "packed:--packed-table" "plain2:"; do
  N=${V%%:*}; A=${V#*:}
  timeout -k 10 300 python bench_aux.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline $A > gpurun_out/${T}_c2_$N.json 2> gpurun_out/${T}_c2_$N.err || exit 1
  python -c "import json; j=json.load(open('gpurun_out/${T}_c2_$N.json')); print('c2 $N', round(j['roofline']['avg_kernel_ms'],3))"
done
