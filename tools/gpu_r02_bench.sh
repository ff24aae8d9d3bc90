# One bench line per configuration and precision into gpurun_out/r02/ (committed under profiles/r02/configs).
set -e
mkdir -p gpurun_out/r02
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r02/bench_$n.json 2> gpurun_out/r02/bench_$n.err
  python -c "import json; d=json.load(open('gpurun_out/r02/bench_$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('prox_hbm'), (d.get('cpu_baseline') or {}).get('value'))"
}
for c in ${CONFIGS:-metric cfg1 cfg2 cfg3 cfg4}; do run $c --config $c; done
run cfg1_latency --config cfg1 --profile 0 --no-cpu-baseline --steps 200 --warmup 10
run cfg2_latency --config cfg2 --profile 0 --no-cpu-baseline --steps 200 --warmup 10
run cfg4_fp16 --config cfg4 --precision fp16 --no-cpu-baseline --steps 10
run cfg4_fp16w2 --config cfg4 --precision fp16w2 --no-cpu-baseline --steps 10
run metric_fp32 --precision fp32 --steps 5 --warmup 1 --no-cpu-baseline
run metric_fp16w2 --precision fp16w2 --steps 10 --no-cpu-baseline
run cfg5 --config cfg5 --steps 3 --warmup 1
