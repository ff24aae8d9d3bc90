#!/bin/bash
# r05 run 16: HEAD mode with its fp32 input ring two steps ahead (LDS-DMA)
set -o pipefail
O=gpurun_out/r05/run16
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_denoiser.py \
  -k "head_tail_inside or two_layers_per_launch" > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 tools/prof_denoise.py --batch 256 \
    > $O/prof.log 2>&1 || exit 1
