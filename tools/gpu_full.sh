# Full GPU test suite, then an A/B of abl_libs (kernel times).
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/full_pytest.log 2>&1 || { tail -30 gpurun_out/full_pytest.log; exit 1; }
tail -2 gpurun_out/full_pytest.log
KFILT=${KFILT:-zzz} bash tools/ab_libs.sh
