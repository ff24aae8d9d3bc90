# cfg2 lines after the head moved into the stack (B = 1): the profiled bench line and the latency line
set -e
mkdir -p gpurun_out/r04/configs
timeout -k 10 300 python3 -u bench.py --config cfg2 > gpurun_out/r04/configs/bench_cfg2.json 2> gpurun_out/r04/configs/bench_cfg2.err
python3 -c "import json; d=json.load(open('gpurun_out/r04/configs/bench_cfg2.json')); print('cfg2', d['value'], d['ms_per_step'])"
timeout -k 10 120 python3 -u bench.py --config cfg2 --profile 0 --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/r04/configs/bench_cfg2_latency.json 2>/dev/null
python3 -c "import json; d=json.load(open('gpurun_out/r04/configs/bench_cfg2_latency.json')); print('cfg2 latency', d['ms_per_step'])"
