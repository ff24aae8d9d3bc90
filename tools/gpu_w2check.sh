set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_denoiser.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/w2_den.log 2>&1 || { tail -30 gpurun_out/w2_den.log; exit 1; }
tail -1 gpurun_out/w2_den.log
timeout -k 10 300 python -u tools/long_parity_probe.py C_rs_3000 A_blur_1200 fp16w2,fp32
timeout -k 10 300 python -u bench.py --config cfg4 --precision fp16w2 --no-cpu-baseline > gpurun_out/w2_cfg4.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/w2_cfg4.json')); print('cfg4 w2', d['value'], d['ms_per_step'], d['kernel_ms'])"
timeout -k 10 300 python -u bench.py --precision fp16w2 --no-cpu-baseline --steps 10 > gpurun_out/w2_metric.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/w2_metric.json')); print('metric w2', d['value'], d['ms_per_step'], d['kernel_ms'])"
