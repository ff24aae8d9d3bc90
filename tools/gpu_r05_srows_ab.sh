#!/bin/bash
# r05: H + 1 rows per strip vs the previous build (8 ceil((H+1)/8)), alternating benches on one box
set -o pipefail
O=gpurun_out/r05/srows_ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --converge-run 0 --no-cpu-baseline > $O/bench_new_$i.json 2> $O/bench_new_$i.err || exit 2
  PNP_LIB_PATH=$GRAFT_REPO_ROOT/abl_libs/conv_head.so timeout -k 10 300 python -u bench.py --converge-run 0 --no-cpu-baseline > $O/bench_old_$i.json 2> $O/bench_old_$i.err || exit 2
done
