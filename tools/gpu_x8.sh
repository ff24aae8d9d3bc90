# 16x16x32 two-layer kernel: accuracy vs the fp16-emulating oracle (the bit-identity test vs one-layer launches
# is expected to fail until the one-layer kernel uses the same K order), then timing
timeout -k 10 300 python -u -m pytest tests/test_gpu_denoiser.py -q -m gpu --timeout 120 --timeout-method thread -k "golden or full_size or ragged" > gpurun_out/x8_pytest.log 2>&1; tail -3 gpurun_out/x8_pytest.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_denoiser.py -q -m gpu --timeout 120 --timeout-method thread -k "two_layers" > gpurun_out/x8_pytest2.log 2>&1; grep -E "passed|failed|Mismatch|Max abs" gpurun_out/x8_pytest2.log | head -12
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/x8_bench.json 2>gpurun_out/x8_bench.err && python -c "import json; d=json.load(open('gpurun_out/x8_bench.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['psnr_img0_db'])"
