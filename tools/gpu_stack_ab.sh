# A/B of the persistent denoiser's halo path: abl_libs/stk_reg.so vs stk_dma.so (tests + B = 1 latency)
set -e
mkdir -p gpurun_out/r03
PNP_LIB_PATH=$PWD/abl_libs/stk_dma.so timeout -k 10 300 python -u -m pytest tests/test_gpu_denoiser.py tests/test_gpu_graph.py -x -q -m gpu --timeout 120 --timeout-method thread -k "one_launch or stack" > gpurun_out/r03/stack_dma_tests.log 2>&1 || { tail -30 gpurun_out/r03/stack_dma_tests.log; exit 1; }
tail -1 gpurun_out/r03/stack_dma_tests.log
for L in stk_reg stk_dma stk_reg stk_dma; do
  PNP_LIB_PATH=$PWD/abl_libs/$L.so timeout -k 10 120 python -u bench.py --config cfg2 --no-cpu-baseline --profile 0 --steps 200 --warmup 20 > gpurun_out/r03/lat_$L.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/r03/lat_$L.json')); print('$L cfg2', d['ms_per_step'])"
done
