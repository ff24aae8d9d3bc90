#!/bin/bash
# r05 run 8: HEAD mode with every wave on L0 and a share of the head
set -o pipefail
O=gpurun_out/r05/run8
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_denoiser.py \
  -k "head_tail_inside or two_layers_per_launch" > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/prof_f1 -o run -- python3 tools/prof_denoise.py --fuse-ends 1 \
    > $O/prof_f1.log 2>&1 || exit 1
