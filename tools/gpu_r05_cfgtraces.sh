#!/bin/bash
# r05: rocprofv3 kernel-trace summaries of each configuration's bench command (short runs)
set -o pipefail
O=gpurun_out/r05/cfgtraces
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in cfg1 cfg2 cfg3 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o trace_$c --output-format csv -- python3 bench.py --config $c \
    --steps 10 --warmup 2 --no-cpu-baseline --converge-run 0 > $O/trace_$c.log 2>&1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O -o trace_cfg5 --output-format csv -- python3 bench.py --config cfg5 \
    --steps 2 --warmup 1 --no-cpu-baseline --converge-run 0 > $O/trace_cfg5.log 2>&1 || exit 1
rm -f $O/*_kernel_trace.csv
