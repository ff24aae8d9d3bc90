# Round-2 check: GPU tests, then one bench line per configuration (metric fp16 / fp32, cfg1-cfg5).
set -e
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest tests/ -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/r02/pytest.log 2>&1 || { tail -40 gpurun_out/r02/pytest.log; exit 1; }
tail -1 gpurun_out/r02/pytest.log
grep -E "max\|dPSNR\||fp32 path" gpurun_out/r02/pytest.log || true
for c in ${CONFIGS:-metric cfg1 cfg2 cfg3 cfg4}; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/r02/bench_$c.json 2> gpurun_out/r02/bench_$c.err
  python -c "import json; d=json.load(open('gpurun_out/r02/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('prox_hbm'), d.get('cpu_baseline',{}).get('value'))"
done
timeout -k 10 400 python -u bench.py --config cfg5 --steps 3 --warmup 1 > gpurun_out/r02/bench_cfg5.json 2> gpurun_out/r02/bench_cfg5.err
python -c "import json; d=json.load(open('gpurun_out/r02/bench_cfg5.json')); print('cfg5', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('cpu_baseline'))"
timeout -k 10 400 python -u bench.py --precision fp32 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02/bench_metric_fp32.json 2> gpurun_out/r02/bench_metric_fp32.err
python -c "import json; d=json.load(open('gpurun_out/r02/bench_metric_fp32.json')); print('fp32', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('roofline'))"
