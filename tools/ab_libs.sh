# A/B of library builds (profiling): bench kernel times per .so under abl_libs/, two rounds.
for round in 1 2; do
for L in ${LIBS:-abl_libs/*.so}; do
  PNP_LIB_PATH=$PWD/$L timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline ${BARGS} 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print('$L', d['value'], {a: round(b, 4) for a, b in k.items() if '${KFILT:-x}' not in a})" || exit 1
done
done
