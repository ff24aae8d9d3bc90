#!/bin/bash
# r05 run 1: the whole GPU suite (with the measured numbers printed), the metric bench, the
# converge full-run bench, and the K2 ablation legs (profiling build).  Test failures (pytest
# rc 1) do not stop the benches; a timeout, crash or fault does.
set -o pipefail
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > $O/bench_metric.json 2> $O/bench_metric.err &&
timeout -k 10 400 python -u bench.py --precision converge --full-run --steps 1200 --warmup 12 --no-cpu-baseline > $O/bench_converge.json 2> $O/bench_converge.err &&
for a in 0 1 2 4 8 16 3 6 7 9 20; do
  PNP_LIB_PATH=pnp-pds_amd/lib_prof/libpnppds.so timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --ablate-k2 $a > $O/k2abl_$a.json 2> $O/k2abl_$a.err || exit 1
done
exit $rc
