# conv_body (variant 1) ablation on the bench workload: profiling only (results are wrong).
# bit0 skip prefetch DMA, bit1 skip stores, bit2 skip MFMA loop
for ab in 0 1 2 3 4 6; do
  PNPPDS_ABLATE=$ab timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --variant 1 > gpurun_out/abl_${ab}.json 2>/dev/null || exit 21
  python -c "import json;d=json.load(open('gpurun_out/abl_${ab}.json'));print('ablate=$ab body_ms',d['kernel_ms']['conv_body'])"
done
