# Two bench ranks on one GPU (gloo barrier/max): exercises bench.py's N>1 path end to end.
export PNP_BENCH_REHEARSAL=1 MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --batch 64 > gpurun_out/rehearse_n2.json 2> gpurun_out/rehearse_n2.err
rc=$?; cat gpurun_out/rehearse_n2.json; tail -3 gpurun_out/rehearse_n2.err; exit $rc
