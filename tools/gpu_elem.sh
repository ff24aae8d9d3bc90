# elementwise K1/K2 (Id, random_sampling operators): parity tests + bench kernel times
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_iter.py tests/test_gpu_cmp.py tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_driver.py > gpurun_out/pt_elem.log 2>&1 || { tail -30 gpurun_out/pt_elem.log; exit 1; }
tail -1 gpurun_out/pt_elem.log
for op in ${OPS:-Id random_sampling}; do timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline --op $op 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print(d['config']['deg_op'], d['value'], k['k1_primal_pre'], k['k2_dual'], k['k3_dual'], d['prox_hbm'])"; done
