# GPU test suite (one process) + smoke, logs under gpurun_out/
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests/ -x -v -s -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
grep -E "max\|dPSNR\||fp32 path|c_n final" gpurun_out/pytest_gpu.log || true
