set -e
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ssim.py > gpurun_out/pt_ssim.log 2>&1 || { tail -30 gpurun_out/pt_ssim.log; exit 1; }
tail -1 gpurun_out/pt_ssim.log
for i in 1 2; do timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['ssim_img0'])"; done
