#!/bin/bash
# r05 run 11: SSIM as one resident wave of blocks with the next tile's loads in flight
set -o pipefail
O=gpurun_out/r05/run11
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ssim.py > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --converge-run 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 2
