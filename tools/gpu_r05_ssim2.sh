#!/bin/bash
# r05: SSIM in two LDS phases (24 KiB, 6 blocks per CU) vs the previous build, alternating
set -o pipefail
O=gpurun_out/r05/ssim2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ssim.py tests/test_gpu_iter.py > $O/pytest.txt 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --converge-run 0 --no-cpu-baseline > $O/bench_new_$i.json 2> $O/bench_new_$i.err || exit 2
  PNP_LIB_PATH=$GRAFT_REPO_ROOT/abl_libs/ops_head.so timeout -k 10 300 python -u bench.py --converge-run 0 --no-cpu-baseline > $O/bench_old_$i.json 2> $O/bench_old_$i.err || exit 2
done
