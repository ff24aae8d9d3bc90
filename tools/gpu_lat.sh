# small-grid (latency) variants of K1 / K2: parity + bit-identity tests, then the cfg2 B = 1 trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_iter.py tests/test_gpu_graph.py tests/test_gpu_long.py -k "not long_trajectory or A_blur_1200" > gpurun_out/lat_tests.log 2>&1
rc=$?; tail -2 gpurun_out/lat_tests.log; grep -E "FAIL|Error" gpurun_out/lat_tests.log | head; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_cfg2_trace.sh
timeout -k 10 120 python3 -u bench.py --config cfg2 --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2 latency', d['ms_per_step'])"
