# A/B on one box, B = 1 (cfg2, --profile 0): none (a9344d5) / head in the stack (44f2b6e) / head + tail in the stack (tree)
set -e
for round in 1 2 3; do
for lib in abl_libs/a9344d5.so abl_libs/44f2b6e.so pnp-pds_amd/lib/libpnppds.so; do
PNP_LIB_PATH=$lib timeout -k 10 120 python3 -u bench.py --config cfg2 --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['ms_per_step'])"
done
done
