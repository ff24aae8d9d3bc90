# Round-3 measurements: the default bench with its rocprofv3 kernel trace and PMC passes, then one
# bench line per configuration (and the B = 1 latency lines).  Outputs under gpurun_out/r03/.
set -e
mkdir -p gpurun_out/r03/bench gpurun_out/r03/configs
export TMPDIR=/tmp
[ -n "$SKIP_BENCH" ] || bash tools/gpu_r03_bench.sh
for c in cfg1 cfg2 cfg3 cfg4; do
  timeout -k 10 300 python3 -u bench.py --config $c > gpurun_out/r03/configs/bench_$c.json 2> gpurun_out/r03/configs/bench_$c.err
  python3 -c "import json; d=json.load(open('gpurun_out/r03/configs/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['config']['precision'], d.get('psnr_delta_db_vs_oracle'))"
done
for c in cfg1 cfg2; do
  timeout -k 10 120 python3 -u bench.py --config $c --profile 0 --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/r03/configs/bench_${c}_latency.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/r03/configs/bench_${c}_latency.json')); print('${c} latency', d['ms_per_step'])"
done
timeout -k 10 400 python3 -u bench.py --config cfg5 --steps 3 --warmup 1 > gpurun_out/r03/configs/bench_cfg5.json 2> gpurun_out/r03/configs/bench_cfg5.err
python3 -c "import json; d=json.load(open('gpurun_out/r03/configs/bench_cfg5.json')); print('cfg5', d['value'], d['ms_per_step'])"
