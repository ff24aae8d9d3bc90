# round 4, first GPU call: smoke + the GPU suite (the ADMM_B2_200 golden still being generated is
# deselected), fp16 long-trajectory numbers with the filter-sum weight rounding, the default
# bench, the self-launched 2-rank rehearsal and the B = 1 latency with cooperative stack launches
set -e
mkdir -p gpurun_out/r04
export PYTEST_ARGS='-k "not ADMM_B2_200"'
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke.log 2>&1
tail -1 gpurun_out/r04/smoke.log
timeout -k 10 1000 python -u -m pytest tests/ -x -v -s -m gpu --timeout 300 --timeout-method thread -k "not ADMM_B2_200" > gpurun_out/r04/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r04/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04/pytest_gpu.log
grep -E "max\|dPSNR\|" gpurun_out/r04/pytest_gpu.log || true
timeout -k 10 600 python -u tools/long_parity_probe.py A_blur_1200 A_blur_s0025_1200 A_blur_s0025_a100_1200 B_blur_300 B_blur_1200 ADMM_B2_30 fp16,fp16w2 > gpurun_out/r04/long_fp16.txt 2>&1
cat gpurun_out/r04/long_fp16.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r04/bench.json 2> gpurun_out/r04/bench.err
cat gpurun_out/r04/bench.json
PNP_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 4 --warmup 1 --batch 64 > gpurun_out/r04/rehearse_n2.json 2> gpurun_out/r04/rehearse_n2.err
cat gpurun_out/r04/rehearse_n2.json
timeout -k 10 300 python -u bench.py --config cfg2 --profile 0 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r04/cfg2_lat.json 2> gpurun_out/r04/cfg2_lat.err
cat gpurun_out/r04/cfg2_lat.json
