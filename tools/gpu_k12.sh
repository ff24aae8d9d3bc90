# blur K1/K2: parity tests + bench kernel times (metric and cfg3)
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_iter.py tests/test_gpu_configs.py tests/test_gpu_cmp.py tests/test_gpu_long.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/k12_pytest.log 2>&1 || { tail -40 gpurun_out/k12_pytest.log; exit 1; }
tail -1 gpurun_out/k12_pytest.log
for c in ${CONFIGS:-metric cfg3}; do
timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/k12_$c.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/k12_$c.json')); print('$c', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if 'conv' not in k}, d['prox_hbm'])"
done
