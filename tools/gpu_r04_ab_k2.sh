# A/B: strip-walking K2 (abl_libs/k2sw.so, the product) vs k2_blur_rb (abl_libs/k2old.so) at the metric / cfg3
set -e
for r in 1 2; do for L in k2sw k2old; do for c in metric cfg3; do
PNP_LIB_PATH=$PWD/abl_libs/$L.so timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print('$L $c', d['value'], k.get('k2_dual'), d['prox_hbm'].get('k2_dual'))"
done; done; done
