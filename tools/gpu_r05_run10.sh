#!/bin/bash
# r05 run 10: whole GPU suite with the head / tail inside the pair launches, the default bench
# (with its converge full-run), smoke
set -o pipefail
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_run10.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > $O/bench_run10.json 2> $O/bench_run10.err || exit 2
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_run10.log 2>&1 || exit 3
exit $rc
