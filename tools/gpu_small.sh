# small-batch (B = 1) iteration latency: cfg1 / cfg2, one- vs two-layer body launches
set -e
for c in cfg1 cfg2; do for L in 1 2; do
timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 50 --warmup 5 --body-layers $L > gpurun_out/small_${c}_$L.json 2>gpurun_out/small_${c}_$L.err
python -c "import json; d=json.load(open('gpurun_out/small_${c}_$L.json')); print('$c L$L', d['value'], d['ms_per_step'], d['kernel_ms'])"
done; done
