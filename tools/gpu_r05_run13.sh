#!/bin/bash
# r05 run 13: the timed region with events around the body launches only
set -o pipefail
O=gpurun_out/r05/run13
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_iter.py -k profile_modes > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --converge-run 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 2
for c in cfg1 cfg2 cfg3; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 3
done
