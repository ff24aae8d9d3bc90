# two split-fp16 layers per hand-off in the B = 1 stack (cfg1): the GPU suite, then a same-box A/B of cfg1 latency
set -e
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_s3x2.log 2>&1 || { grep -E "PASS|FAIL|Error|assert|^E " gpurun_out/r04/pytest_s3x2.log | tail -40; exit 1; }
tail -2 gpurun_out/r04/pytest_s3x2.log
for round in 1 2 3; do
for lib in abl_libs/base.so pnp-pds_amd/lib/libpnppds.so; do
PNP_LIB_PATH=$lib timeout -k 10 120 python3 -u bench.py --config cfg1 --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg1 $lib', d['ms_per_step'])"
done
done
