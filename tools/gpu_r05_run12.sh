#!/bin/bash
# r05 run 12: cfg5 (comparisonB-2, 64 x RGB 1024^2; a step is one outer iteration)
set -o pipefail
O=gpurun_out/r05/configs
mkdir -p $O
timeout -k 10 600 python -u bench.py --config cfg5 --steps 3 --warmup 1 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || exit 1
