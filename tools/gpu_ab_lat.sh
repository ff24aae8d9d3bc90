# A/B of library builds without per-kernel events (--profile 0: the unprofiled launch sequence):
# ms per iteration for each .so under abl_libs/ at the configs in CFGS, two rounds.
set -e
for round in 1 2; do
for c in ${CFGS:-metric cfg2}; do
for L in ${LIBS:-abl_libs/*.so}; do
  if [ "$c" = metric ]; then A="--steps 20 --warmup 3"; else A="--steps 300 --warmup 30"; fi
  PNP_LIB_PATH=$PWD/$L timeout -k 10 200 python -u bench.py --config $c --profile 0 $A --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $L', d['value'], d['ms_per_step'])"
done
done
done
