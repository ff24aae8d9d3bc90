# l1_select packed/replicated LDS bins: parity tests (product library), then A/B at cfg3 and cfg5 (profiling).
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_cmp.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/l1_pytest.log 2>&1 || { tail -30 gpurun_out/l1_pytest.log; exit 1; }
tail -1 gpurun_out/l1_pytest.log
BARGS="--config cfg3" KFILT=conv bash tools/ab_libs.sh
BARGS="--config cfg5 --steps 1 --warmup 1" KFILT=conv bash tools/ab_libs.sh
