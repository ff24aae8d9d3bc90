# SSIM / K2 checks: parity tests + bench kernel times
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_iter.py tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_cmp.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ssim_pytest.log 2>&1 || { tail -40 gpurun_out/ssim_pytest.log; exit 1; }
tail -1 gpurun_out/ssim_pytest.log
for c in ${CONFIGS:-metric}; do
for op in blur random_sampling; do
timeout -k 10 300 python -u bench.py --config $c --op $op --no-cpu-baseline > gpurun_out/ssim_$c$op.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/ssim_$c$op.json')); print('$c $op', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if 'conv' not in k}, d['ssim_img0'])"
done; done
