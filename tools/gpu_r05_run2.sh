#!/bin/bash
# r05 run 2: the whole GPU suite after the fp32 K2 epilogue, fp16a2 stacks and tolerance overrides;
# the metric bench twice (box-to-box / run-to-run spread of K2 and the CPU baseline)
set -o pipefail
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_run2.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > $O/bench_metric2.json 2> $O/bench_metric2.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_metric3.json 2> $O/bench_metric3.err
r2=$?; [ $r2 -ne 0 ] && exit $r2
exit $rc
