# XCD-aware tile order of the blur passes: operator/iteration tests, then A/B of abl_libs (kernel times)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_iter.py tests/test_gpu_graph.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/xcd_tests.log 2>&1 || { tail -40 gpurun_out/xcd_tests.log; exit 1; }
tail -1 gpurun_out/xcd_tests.log
BARGS0="--steps 10" KFILT=conv bash tools/gpu_ab.sh
BARGS0="--steps 10" KFILT=conv CFGS=cfg3 bash tools/gpu_ab.sh
