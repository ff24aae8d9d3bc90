# Late r02: pass-split + config tests, then the fp32 lines and cfg5's line with HBM-sized denoiser passes.
set -e
mkdir -p gpurun_out/r02
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_configs.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/late_pytest.log 2>&1 || { tail -30 gpurun_out/late_pytest.log; exit 1; }
tail -1 gpurun_out/late_pytest.log
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r02/bench_$n.json 2> gpurun_out/r02/bench_$n.err
  python -c "import json; d=json.load(open('gpurun_out/r02/bench_$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('kernel_calls_per_step'))"
}
run cfg5 --config cfg5 --steps 3 --warmup 1
run cfg4 --config cfg4
run metric_fp32 --precision fp32 --steps 5 --warmup 1 --no-cpu-baseline
