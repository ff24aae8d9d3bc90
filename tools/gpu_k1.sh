# K1 fill variants: parity (product library), then A/B of abl_libs (K1/K2 times)
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_iter.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/k1_pytest.log 2>&1; tail -2 gpurun_out/k1_pytest.log
KFILT=conv bash tools/ab_libs.sh
