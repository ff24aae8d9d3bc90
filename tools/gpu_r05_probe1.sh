#!/bin/bash
# r05 probe 1: c_n fidelity of fp16 -> split-fp16 hand-over at K iterations / at a c_n threshold;
# baseline bench
set -o pipefail
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 python -u tools/converge_probe.py A_blur_1200 fp16 fp16x3 0 2 3 5 8 12 16 1200 > $O/conv_A.txt 2>&1 &&
timeout -k 10 300 python -u tools/converge_probe.py A_blur_1200 auto converge 10000 5000 3000 2000 1000 >> $O/conv_A.txt 2>&1 &&
timeout -k 10 300 python -u tools/converge_probe.py B_blur_1200 fp16 fp16x3 0 20 50 80 104 1200 > $O/conv_B.txt 2>&1 &&
timeout -k 10 300 python -u tools/converge_probe.py B_blur_1200 auto converge 10000 5000 3000 >> $O/conv_B.txt 2>&1 &&
timeout -k 10 300 python -u tools/converge_probe.py ADMM_B2_200 fp16 fp16x3 0 5 10 13 200 > $O/conv_ADMM.txt 2>&1 &&
timeout -k 10 300 python -u tools/converge_probe.py ADMM_B2_200 auto converge 10000 3000 >> $O/conv_ADMM.txt 2>&1 &&
timeout -k 10 300 python -u tools/converge_probe.py A_blur_1200 fp16w2 fp16x3 1200 > $O/conv_A_w2.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench0.json 2> $O/bench0.err
