#!/bin/bash
# r05 run 14: stack rooflines for B = 1; the metric with and without the body-launch events
set -o pipefail
O=gpurun_out/r05/run14
mkdir -p $O
for c in cfg1 cfg2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 3
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --converge-run 0 --no-cpu-baseline > $O/bench_ev_$i.json 2> $O/bench_ev_$i.err || exit 2
  timeout -k 10 300 python -u bench.py --converge-run 0 --no-cpu-baseline --profile 0 > $O/bench_noev_$i.json 2> $O/bench_noev_$i.err || exit 2
done
