# persistent small-batch denoiser: bit-identity tests + B = 1 latency (cfg2 fp16, cfg1 x3)
set -e
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_denoiser.py tests/test_gpu_graph.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03/stack_tests.log 2>&1 || { tail -30 gpurun_out/r03/stack_tests.log; exit 1; }
tail -1 gpurun_out/r03/stack_tests.log
for bl in 1 0; do
  timeout -k 10 120 python -u bench.py --config cfg2 --no-cpu-baseline --profile 0 --steps 200 --warmup 20 --body-layers $bl > gpurun_out/r03/lat_cfg2_bl$bl.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/r03/lat_cfg2_bl$bl.json')); print('cfg2 body_layers=$bl', d['ms_per_step'], d['value'])"
done
timeout -k 10 120 python -u bench.py --config cfg2 --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/r03/prof_cfg2.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/r03/prof_cfg2.json')); print(d['kernel_ms'])"
for bl in 1 0; do
  timeout -k 10 120 python -u bench.py --config cfg1 --no-cpu-baseline --profile 0 --steps 100 --warmup 10 --body-layers $bl > gpurun_out/r03/lat_cfg1_bl$bl.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/r03/lat_cfg1_bl$bl.json')); print('cfg1 body_layers=$bl', d['ms_per_step'], d['value'], d['config']['precision'])"
done
