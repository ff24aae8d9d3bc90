#!/bin/bash
# r05: the N > 1 bench path rehearsed with two ranks on one GPU (gloo), under torch.distributed.run and self-launched
set -o pipefail
O=gpurun_out/r05/rehearse
mkdir -p $O
export PNP_BENCH_REHEARSAL=1 MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --batch 64 > $O/torchrun.json 2> $O/torchrun.err || exit 1
timeout -k 10 300 python bench.py --gpus 2 --steps 4 --warmup 1 --batch 64 > $O/self_launch.json 2> $O/self_launch.err || exit 2
