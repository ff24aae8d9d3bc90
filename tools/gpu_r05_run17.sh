#!/bin/bash
# r05 run 17 (diagnostic, results wrong in the variants): what bounds the HEAD-mode launch
set -o pipefail
O=gpurun_out/r05/run17
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in product x8h_nohead x8h_nol0 x8p_nol; do
  if [ $v = product ]; then L=""; else L="$GRAFT_REPO_ROOT/abl_libs/$v.so"; fi
  PNP_LIB_PATH=$L timeout -k 10 240 rocprofv3 --kernel-trace -d $O/prof_$v -o run -- python3 tools/prof_denoise.py --batch 256 \
    > $O/prof_$v.log 2>&1 || exit 1
done
