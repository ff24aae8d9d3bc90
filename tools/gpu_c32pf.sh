# fp32 body halo prefetch: fp32 tests with the product library, then A/B of abl_libs at fp32.
timeout -k 10 600 python -u -m pytest tests/test_gpu_denoiser.py tests/test_gpu_configs.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/c32pf.log 2>&1 || { tail -40 gpurun_out/c32pf.log; exit 1; }
tail -2 gpurun_out/c32pf.log
BARGS="--precision fp32 --steps 3 --warmup 1" KFILT=zzz bash tools/ab_libs.sh
