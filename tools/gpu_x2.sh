# conv_stack16x2 (two body layers per hand-off): bit-identity tests, then cfg2 B = 1 latency (3 = pairs, 4 = one per hand-off)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_denoiser.py -k "all_layers" tests/test_gpu_graph.py > gpurun_out/x2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/x2_tests.log; grep -E "FAIL|Error" gpurun_out/x2_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
for bl in 4 3 4 3; do
  timeout -k 10 120 python3 -u bench.py --config cfg2 --profile 0 --steps 300 --warmup 30 --no-cpu-baseline --body-layers $bl 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2 body-layers $bl', d['ms_per_step'])" || exit 1
done
timeout -k 10 120 python3 -u bench.py --config cfg2 --steps 100 --warmup 10 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2 profiled', d['ms_per_step'], d['kernel_ms'])"
