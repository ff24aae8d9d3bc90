#!/bin/bash
# r05 final: whole GPU suite, smoke, the default bench line, then the profile of the bench command
set -o pipefail
O=gpurun_out/r05/final
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 4
exit $rc
