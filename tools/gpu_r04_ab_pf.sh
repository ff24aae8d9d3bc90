# A/B: the B = 1 stack's B-fragment prefetch depth (abl_libs/pf{1,2,3}.so), cfg2 / cfg1 latency
set -e
for r in 1 2; do for L in pf1 pf2 pf3; do for c in cfg2; do
PNP_LIB_PATH=$PWD/abl_libs/$L.so timeout -k 10 200 python -u bench.py --config $c --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L $c', d['ms_per_step'], d['value'])"
done; done; done
