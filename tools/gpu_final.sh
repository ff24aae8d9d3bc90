# Round-end: GPU tests, smoke, then the bench profile (trace + PMC passes) into gpurun_out/prof_final.
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/final_pytest.log 2>&1 || { tail -30 gpurun_out/final_pytest.log; exit 1; }
tail -2 gpurun_out/final_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
bash tools/profile_bench.sh gpurun_out/prof_final
