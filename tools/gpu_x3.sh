# fp16x3 (split fp16) first check: denoiser parity, long trajectories, bench at the metric / cfg4
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_denoiser.py tests/test_gpu_long.py -x -v -s -m gpu --timeout 300 --timeout-method thread -k "fp16x3 and not gray" > gpurun_out/x3_tests.log 2>&1 || { tail -40 gpurun_out/x3_tests.log; exit 1; }
grep -E "max\|d|dPSNR|passed|failed" gpurun_out/x3_tests.log || true
timeout -k 10 300 python -u bench.py --precision fp16x3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/x3_metric.json 2> gpurun_out/x3_metric.err
timeout -k 10 300 python -u bench.py --config cfg4 --precision fp16x3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/x3_cfg4.json 2> gpurun_out/x3_cfg4.err
python -c "
import json
for f in ('x3_metric','x3_cfg4'):
    d=json.loads(open('gpurun_out/'+f+'.json').read())
    print(f, d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('kernel_ms'))
"
