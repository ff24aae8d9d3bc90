# split head inside the fp16x3 stack (cfg1, B = 1): the GPU suite, then a same-box A/B of cfg1 latency
set -e
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_s3head.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/r04/pytest_s3head.log | tail -30; exit 1; }
tail -2 gpurun_out/r04/pytest_s3head.log
for round in 1 2 3; do
for lib in abl_libs/61af447.so pnp-pds_amd/lib/libpnppds.so; do
PNP_LIB_PATH=$lib timeout -k 10 120 python3 -u bench.py --config cfg1 --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg1 $lib', d['ms_per_step'])"
done
done
