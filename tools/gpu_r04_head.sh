# head layer computed inside the two-layer stack (B = 1): bit-identity tests, the long goldens, cfg2 latency
set -e
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_denoiser.py tests/test_gpu_long.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_head.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/r04/pytest_head.log | tail -30; exit 1; }
tail -2 gpurun_out/r04/pytest_head.log
for i in 1 2 3; do
timeout -k 10 120 python3 -u bench.py --config cfg2 --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2 latency', d['ms_per_step'])"
done
timeout -k 10 120 python3 -u bench.py --config cfg2 --steps 50 --warmup 10 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2 kernels', d.get('kernel_ms'))"
