# Register-blocked standalone blur operator (k0_blur_rb): parity tests (product library), then A/B at cfg5 (profiling).
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_cmp.py tests/test_gpu_iter.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/k0_pytest.log 2>&1 || { tail -30 gpurun_out/k0_pytest.log; exit 1; }
tail -1 gpurun_out/k0_pytest.log
BARGS="--config cfg5 --steps 1 --warmup 1" KFILT=conv bash tools/ab_libs.sh
