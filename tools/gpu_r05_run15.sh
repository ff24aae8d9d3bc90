#!/bin/bash
# r05 run 15: the configuration tests' measured deviations from the oracle (for their tolerances)
set -o pipefail
O=gpurun_out/r05/run15
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_long.py -k "cfg or metric_batch" > $O/pytest.txt 2>&1
