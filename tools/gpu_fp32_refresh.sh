# Refresh the fp32-operand bench lines (cfg4's default precision, and the metric at fp32) into gpurun_out/r02/.
set -e
mkdir -p gpurun_out/r02
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r02/bench_$n.json 2> gpurun_out/r02/bench_$n.err
  python -c "import json; d=json.load(open('gpurun_out/r02/bench_$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('roofline'))"
}
run cfg4 --config cfg4
run metric_fp32 --precision fp32 --steps 5 --warmup 1 --no-cpu-baseline
