# round 4, GPU call 3: the suite on the strip-walking K2 + side-stream SSIM, the K2 and stack-prefetch
# A/Bs, then the profile (bench trace + PMC passes + configs)
set -e
mkdir -p gpurun_out/r04
timeout -k 10 1000 python -u -m pytest tests/ -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r04/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04/pytest_gpu.log
grep -E "max\|dPSNR\|" gpurun_out/r04/pytest_gpu.log | grep -E "auto" || true
bash tools/gpu_r04_ab_k2.sh
bash tools/gpu_r04_ab_pf.sh
SKIP_TESTS=1 bash tools/gpu_r04_profile.sh
