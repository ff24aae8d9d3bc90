set -e
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -x -v -s -m gpu --timeout 600 --timeout-method thread > gpurun_out/r03/cfgtests.log 2>&1 || { tail -30 gpurun_out/r03/cfgtests.log; exit 1; }
grep -E "passed|failed|cfg5 crop" gpurun_out/r03/cfgtests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03/bench_metric_quick.json 2> gpurun_out/r03/bench_metric_quick.err
python -c "
import json; d=json.load(open('gpurun_out/r03/bench_metric_quick.json')); print(d['value'], d['hbm_copy_gbs'], d['prox_hbm'], d['roofline']['frac'])"
