# Round-2 close: the driver's order (smoke, GPU tests, default bench), then the bench profile refresh.
set -e
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1; tail -1 gpurun_out/fin_smoke.log
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1 || { tail -30 gpurun_out/fin_pytest.log; exit 1; }
tail -1 gpurun_out/fin_pytest.log
timeout -k 10 400 python -u bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err; cat gpurun_out/fin_bench.json
bash tools/profile_bench.sh gpurun_out/prof_fin
