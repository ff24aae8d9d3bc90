set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_denoiser.py tests/test_gpu_long.py -x -q -m gpu --timeout 300 --timeout-method thread -k "fp16x3 and not gray" > gpurun_out/x3_tests.log 2>&1 || { tail -40 gpurun_out/x3_tests.log; exit 1; }
tail -1 gpurun_out/x3_tests.log
CFGS="metric cfg4" BARGS0="--precision fp16x3 --warmup 2" bash tools/gpu_ab.sh
