set -e
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_denoiser.py > gpurun_out/pt_den.log 2>&1 || { tail -30 gpurun_out/pt_den.log; exit 1; }
tail -1 gpurun_out/pt_den.log
timeout -k 10 200 python -u tools/ab_body.py ${ABARGS:---variants 0,2} --rounds 5 2>&1 | grep variant
