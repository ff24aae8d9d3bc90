# fused two-layer body kernel: bit-identity tests first, then the bench (metric) with both settings
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_denoiser.py -x -q -m gpu --timeout 120 --timeout-method thread -k "two_layers or golden or full_size" > gpurun_out/f2_pytest.log 2>&1 || { tail -40 gpurun_out/f2_pytest.log; exit 1; }
tail -1 gpurun_out/f2_pytest.log
for L in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --body-layers $L > gpurun_out/f2_bench$L.json 2>gpurun_out/f2_bench$L.err
python -c "import json; d=json.load(open('gpurun_out/f2_bench$L.json')); print('layers $L metric', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
