set -e
timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/bk.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/bk.json')); k=d['kernel_ms']; print(d['value'], k, d['prox_hbm'], d['psnr_img0_db'])"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_iter.py tests/test_gpu_cmp.py tests/test_gpu_ops.py tests/test_gpu_configs.py > gpurun_out/pt_k12.log 2>&1
tail -1 gpurun_out/pt_k12.log
