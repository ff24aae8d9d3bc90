# x8 dead-group skip: bit-identity tests of the body with the product build, then A/B (kernel times)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_denoiser.py tests/test_gpu_iter.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/skip_tests.log 2>&1 || { tail -30 gpurun_out/skip_tests.log; exit 1; }
tail -1 gpurun_out/skip_tests.log
BARGS0="--steps 20" KFILT=k_ bash tools/gpu_ab.sh
