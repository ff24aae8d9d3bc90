#!/bin/bash
# r05 run 7: head / tail inside the pair launches (PNP_TUNE_FUSE_ENDS): bit-identity, then the
# denoiser's kernel times fused vs apart, then the default bench
set -o pipefail
O=gpurun_out/r05/run7
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_denoiser.py \
  -k "head_tail_inside or two_layers_per_launch or golden" > $O/pytest.txt 2>&1 || exit 1
for f in 1 0; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_f$f -o run -- python3 tools/prof_denoise.py --fuse-ends $f \
    > $O/prof_f$f.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
