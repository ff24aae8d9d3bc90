#!/bin/bash
# r05 diagnostic: the two-layer launch's time per image row at H = 256 (strips padded to 264 rows)
# vs H = 255 (256 = H + 1: no padding step)
set -o pipefail
O=gpurun_out/r05/pad
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for h in 256 255 256 255; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d $O/prof_$h -o run -- python3 tools/prof_denoise.py --batch 256 --height $h \
    > $O/prof_$h.log 2>&1 || exit 1
  python3 tools/rocpd_stats.py $O/prof_$h/run_results.db conv_body >> $O/summary_$h.txt
  rm -rf $O/prof_$h
done
