# round-4 close: the fp32 numbers of the two ill-conditioned sigma-0.04 goldens, the whole GPU
# suite under the sigma-aware auto policy, the default bench line, cfg2 latency per precision
set -e
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u tools/long_parity_probe.py B_blur_s004_1200 FBS_blur_s004_1200 fp32,fp16x3 > gpurun_out/r04/long_grid3.txt 2>&1 || { tail -40 gpurun_out/r04/long_grid3.txt; exit 1; }
cat gpurun_out/r04/long_grid3.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_all.log 2>&1 || { grep -E "max\|dPSNR\||pixels off|PASS|FAIL|Error" gpurun_out/r04/pytest_all.log | tail -30; tail -30 gpurun_out/r04/pytest_all.log; exit 1; }
grep -E "max\|dPSNR\||pixels off" gpurun_out/r04/pytest_all.log
tail -3 gpurun_out/r04/pytest_all.log
timeout -k 10 600 python -u bench.py > gpurun_out/r04/bench_final.json 2> gpurun_out/r04/bench_final.err
cat gpurun_out/r04/bench_final.json
for p in fp16 fp16w2 fp16x3; do
timeout -k 10 120 python3 -u bench.py --config cfg2 --precision $p --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2 latency $p', d['ms_per_step'])"
done
timeout -k 10 300 python3 -u bench.py --precision fp16w2 --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('metric fp16w2', d['value'], d['ms_per_step'])"
