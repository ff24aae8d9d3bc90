set -e
mkdir -p gpurun_out/r03
PNP_LIB_PATH=$PWD/abl_libs/x8_clock.so timeout -k 10 180 python3 -u tools/x8_clock.py
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r03/copycheck.json 2>/dev/null
python3 -c "import json; d=json.load(open('gpurun_out/r03/copycheck.json')); print('copy', d['hbm_copy_gbs'], d['prox_hbm'])"
