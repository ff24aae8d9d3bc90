#!/bin/bash
# r05: the strip stream with H + 1 rows per strip: bit-identity and denoiser tests, then timing
set -o pipefail
O=gpurun_out/r05/srows
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_denoiser.py tests/test_gpu_iter.py \
  > $O/pytest.txt 2>&1 || exit 1
for h in 256 255; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d $O/prof_$h -o run -- python3 tools/prof_denoise.py --batch 256 --height $h \
    > $O/prof_$h.log 2>&1 || exit 1
  python3 tools/rocpd_stats.py $O/prof_$h/run_results.db conv_body > $O/summary_$h.txt
  rm -rf $O/prof_$h
done
