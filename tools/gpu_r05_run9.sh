#!/bin/bash
# r05 run 9: denoiser kernel times at the metric's batch (256), ends fused vs apart
set -o pipefail
O=gpurun_out/r05/run9
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 1 0; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d $O/prof_f$f -o run -- python3 tools/prof_denoise.py --batch 256 --fuse-ends $f \
    > $O/prof_f$f.log 2>&1 || exit 1
done
