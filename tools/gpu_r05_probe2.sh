#!/bin/bash
# r05 probe 2: fp16a2 (split activations, fp16 weights) as the hand-over precision: c_n / PSNR
# on the long goldens, and its speed at the metric beside fp16x3
set -o pipefail
O=gpurun_out/r05
mkdir -p $O
P="timeout -k 10 300 python -u tools/converge_probe.py"
{ $P A_blur_1200 fp16 fp16a2 0 7 && $P B_blur_1200 fp16 fp16a2 0 106 && $P ADMM_B2_200 fp16 fp16a2 0 15 &&
  $P A_blur_s004_1200 fp16w2 fp16a2 0 14 && $P A_blur_s002_1200 fp16w2 fp16a2 0 14 &&
  $P FBS_blur_s004_1200 fp16x3 fp16a2 0 && $P RED_blur_s004_1200 fp16x3 fp16a2 0 && $P B_blur_s004_1200 fp16x3 fp16a2 0 &&
  $P A_blur_s0025_1200 fp16 fp16a2 0 14 && $P C_rs_3000 fp16x3 fp16a2 0 && $P A_rs_3000 fp16x3 fp16a2 0 &&
  $P A_gray_id_1200 fp16x3 fp16a2 0; } > $O/a2_probe.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --precision fp16a2 --no-cpu-baseline > $O/bench_a2.json 2> $O/bench_a2.err &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --precision fp16x3 --no-cpu-baseline > $O/bench_x3.json 2> $O/bench_x3.err
