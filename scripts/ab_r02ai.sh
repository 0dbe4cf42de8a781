set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/make_tierc_fixture.py --out gpurun_out/tierc_c3_seq.json > gpurun_out/r02ai_fixture.log 2>&1 || exit 1
cp gpurun_out/tierc_c3_seq.json tests/golden/tierc_c3_seq.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_tierc.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r02ai_tierc.log 2>&1 || exit 1
