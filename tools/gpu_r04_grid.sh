# main.py's blur grid: fp16 / fp16x3 numbers of the grid goldens (probe), then the goldens under auto (GPU tests)
set -e
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u tools/long_parity_probe.py A_blur_s0005_1200 A_blur_s002_1200 A_blur_s004_1200 A_blur_s0025_a082_1200 FBS_blur_1200 FBS_blur_s0025_1200 RED_blur_1200 RED_blur_s0025_1200 fp16,fp16w2,fp16x3 > gpurun_out/r04/long_grid.txt 2>&1 || { tail -40 gpurun_out/r04/long_grid.txt; exit 1; }
cat gpurun_out/r04/long_grid.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py -v -s --timeout 300 --timeout-method thread -k "s0005 or s002_ or s004 or a082 or FBS or RED" > gpurun_out/r04/pytest_grid.log 2>&1 || true
grep -E "max\|dPSNR\||passed|failed" gpurun_out/r04/pytest_grid.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_denoiser.py -v --timeout 120 --timeout-method thread -k side_stream > gpurun_out/r04/pytest_side.log 2>&1 || true
grep -E "PASS|FAIL|passed|failed" gpurun_out/r04/pytest_side.log
