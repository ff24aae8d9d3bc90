set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_blur_mf.py tests/test_gpu_ops.py tests/test_gpu_iter.py > gpurun_out/mf_tests.log 2>&1
rc=$?; tail -5 gpurun_out/mf_tests.log; grep -E "FAIL|Error|assert" gpurun_out/mf_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/mf_bench.json 2> gpurun_out/mf_bench.err && python -c "import json; d=json.load(open('gpurun_out/mf_bench.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['prox_hbm'])"
