# fp32 denoiser tail on the VALU: its tests, then fp32 timings (metric and cfg4).
timeout -k 10 600 python -u -m pytest tests/test_gpu_denoiser.py tests/test_gpu_configs.py tests/test_gpu_graph.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/fp32tail.log 2>&1 || { tail -40 gpurun_out/fp32tail.log; exit 1; }
tail -2 gpurun_out/fp32tail.log
timeout -k 10 300 python -u bench.py --precision fp32 --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('metric_fp32', d['value'], d['ms_per_step'], d['kernel_ms'])" || exit 1
timeout -k 10 300 python -u bench.py --config cfg4 --steps 5 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4', d['value'], d['ms_per_step'], d['precision'] if 'precision' in d else '', d['kernel_ms'])" || exit 1
