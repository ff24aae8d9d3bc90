# A/B: waves per SIMD of the batched K1 / K2 blur passes (abl_libs/w{66,76,77}.so: K1, K2 occupancy)
set -e
for r in 1 2; do for L in w66 w76 w77; do for c in metric cfg3; do
PNP_LIB_PATH=$PWD/abl_libs/$L.so timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print('$L $c', d['value'], k.get('k1_primal_pre'), k.get('k2_dual'), d['prox_hbm'])"
done; done; done
