set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_iter.py tests/test_gpu_configs.py tests/test_gpu_cmp.py tests/test_gpu_long.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/l1_pytest.log 2>&1 || { tail -40 gpurun_out/l1_pytest.log; exit 1; }
tail -1 gpurun_out/l1_pytest.log
timeout -k 10 300 python -u bench.py --config cfg3 --no-cpu-baseline > gpurun_out/l1_cfg3.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/l1_cfg3.json')); print('cfg3', d['value'], d['ms_per_step'], d['kernel_ms'], d['prox_hbm'])"
