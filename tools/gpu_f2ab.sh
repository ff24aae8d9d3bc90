# fused body: bit-identity tests, then A/B of abl_libs/*.so variants (kernel times, metric)
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_denoiser.py -x -q -m gpu --timeout 120 --timeout-method thread -k "two_layers or golden or full_size" > gpurun_out/f2_pytest.log 2>&1 || { tail -40 gpurun_out/f2_pytest.log; exit 1; }
tail -1 gpurun_out/f2_pytest.log
for L in abl_libs/*.so; do
  PNP_LIB_PATH=$PWD/$L timeout -k 10 120 python -u -m pytest tests/test_gpu_denoiser.py -x -q -m gpu --timeout 120 --timeout-method thread -k "two_layers" > gpurun_out/f2_ab_pytest.log 2>&1 || { echo "$L failed"; tail -30 gpurun_out/f2_ab_pytest.log; exit 1; }
done
KFILT=x bash tools/ab_libs.sh
