# 64 x 32 blur tiles (more blocks per CU) vs 64 x 64: A/B kernel times, then the h32 build's parity tests
set -e
mkdir -p gpurun_out
BARGS0="--steps 10" KFILT=conv bash tools/gpu_ab.sh
PNP_LIB_PATH=$PWD/abl_libs/h32.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_iter.py tests/test_gpu_graph.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/h32_tests.log 2>&1 || { tail -30 gpurun_out/h32_tests.log; exit 1; }
tail -1 gpurun_out/h32_tests.log
PNP_LIB_PATH=$PWD/abl_libs/h32.so timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu -k cfg3 --timeout 300 --timeout-method thread > gpurun_out/h32_cfg3.log 2>&1 || { tail -30 gpurun_out/h32_cfg3.log; exit 1; }
tail -1 gpurun_out/h32_cfg3.log
