# Round-4 measurements: the GPU suite, the default bench with its rocprofv3 kernel trace and PMC
# passes (profile_bench.sh), then one bench line per configuration and the B = 1 latency lines.
# Outputs under gpurun_out/r04/.
set -e
mkdir -p gpurun_out/r04/bench gpurun_out/r04/configs
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests/ -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r04/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/r04/pytest_gpu.log
  grep -E "max\|dPSNR\|" gpurun_out/r04/pytest_gpu.log | grep -E "auto|fp16\)" || true
fi
if [ -z "$SKIP_BENCH" ]; then
  bash tools/profile_bench.sh gpurun_out/r04/bench
  F=$(find gpurun_out/r04/bench -name "pmc_fetch_counter_collection.csv" | head -1)
  W=$(find gpurun_out/r04/bench -name "pmc_write_counter_collection.csv" | head -1)
  python3 tools/traffic_from_pmc.py $F $W --out gpurun_out/r04/bench/traffic.json > /dev/null
  python3 tools/pmc_summary.py $(find gpurun_out/r04/bench -name "pmc_*_counter_collection.csv") > gpurun_out/r04/bench/pmc_summary.txt
  python3 -c "import json; d=json.load(open('gpurun_out/r04/bench/bench.json')); print('metric', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernel_ms'], d.get('prox_hbm'))"
fi
if [ -z "$SKIP_CONFIGS" ]; then
  for c in cfg1 cfg2 cfg3 cfg4; do
    timeout -k 10 300 python3 -u bench.py --config $c > gpurun_out/r04/configs/bench_$c.json 2> gpurun_out/r04/configs/bench_$c.err
    python3 -c "import json; d=json.load(open('gpurun_out/r04/configs/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['config']['precision'], d.get('psnr_delta_db_vs_oracle'))"
  done
  for c in cfg1 cfg2; do
    timeout -k 10 120 python3 -u bench.py --config $c --profile 0 --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/r04/configs/bench_${c}_latency.json 2>/dev/null
    python3 -c "import json; d=json.load(open('gpurun_out/r04/configs/bench_${c}_latency.json')); print('${c} latency', d['ms_per_step'])"
  done
  timeout -k 10 400 python3 -u bench.py --config cfg5 --steps 3 --warmup 1 > gpurun_out/r04/configs/bench_cfg5.json 2> gpurun_out/r04/configs/bench_cfg5.err
  python3 -c "import json; d=json.load(open('gpurun_out/r04/configs/bench_cfg5.json')); print('cfg5', d['value'], d['ms_per_step'])"
fi
