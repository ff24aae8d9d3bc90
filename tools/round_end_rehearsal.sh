# What the driver runs at round end, in order (smoke, GPU tests, default bench)
set -e
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/re_smoke.log 2>&1; tail -1 gpurun_out/re_smoke.log
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/re_pytest.log 2>&1; tail -1 gpurun_out/re_pytest.log
timeout -k 10 400 python -u bench.py > gpurun_out/re_bench.json 2> gpurun_out/re_bench.err; cat gpurun_out/re_bench.json
