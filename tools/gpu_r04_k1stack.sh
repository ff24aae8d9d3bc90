# K1 inside the two-layer stack (B = 1 ours-A on blur_1): the GPU suite, then a same-box A/B of cfg2 latency
set -e
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_k1stack.log 2>&1 || { grep -E "PASS|FAIL|Error|assert|^E " gpurun_out/r04/pytest_k1stack.log | tail -40; exit 1; }
tail -2 gpurun_out/r04/pytest_k1stack.log
for round in 1 2 3; do
for lib in abl_libs/138032f.so pnp-pds_amd/lib/libpnppds.so; do
PNP_LIB_PATH=$lib timeout -k 10 120 python3 -u bench.py --config cfg2 --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg2 $lib', d['ms_per_step'])"
done
done
