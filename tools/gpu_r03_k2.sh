# K2 fill rework + K3 fused into K1: operator/iteration/config/graph GPU tests, then the metric bench
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_iter.py tests/test_gpu_graph.py tests/test_gpu_configs.py tests/test_gpu_long.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/k2_tests.log 2>&1 || { tail -40 gpurun_out/k2_tests.log; exit 1; }
tail -1 gpurun_out/k2_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/k2_bench.json 2> gpurun_out/k2_bench.err
python -c "import json; d=json.load(open('gpurun_out/k2_bench.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['prox_hbm'], d.get('psnr_delta_db_vs_oracle'))"
done
timeout -k 10 200 python -u bench.py --config cfg3 --no-cpu-baseline > gpurun_out/k2_cfg3.json 2> gpurun_out/k2_cfg3.err
python -c "import json; d=json.load(open('gpurun_out/k2_cfg3.json')); print('cfg3', d['value'], d['ms_per_step'], d['kernel_ms'], d['prox_hbm'], d.get('psnr_delta_db_vs_oracle'))"
for c in cfg1 cfg2; do
timeout -k 10 120 python3 -u bench.py --config $c --profile 0 --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/k2_${c}_lat.json 2>/dev/null
python3 -c "import json; d=json.load(open('gpurun_out/k2_${c}_lat.json')); print('${c} latency', d['ms_per_step'])"
done
