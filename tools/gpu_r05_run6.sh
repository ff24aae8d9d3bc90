#!/bin/bash
# r05 run 6: the default bench twice (CPU leg now before the GPU initializes) and the configs
set -o pipefail
O=gpurun_out/r05/configs
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_metric_a.json 2> $O/bench_metric_a.err || exit 1
timeout -k 10 400 python -u bench.py > $O/bench_metric_b.json 2> $O/bench_metric_b.err || exit 1
for c in cfg1 cfg2 cfg3 cfg4; do
  timeout -k 10 400 python -u bench.py --config $c --converge-run 0 > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
timeout -k 10 600 python -u bench.py --config cfg5 --steps 3 --warmup 1 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || exit 1
