#!/bin/bash
# r05 run 3: K2 float32 vs fp64 epilogue A/B on one box (lib_prof, ABL 0 / 32 alternating), the
# tests the K2 change touches, and the two-rank rehearsals (torch.distributed.run and bench.py's
# own launcher) on the one device
set -o pipefail
O=gpurun_out/r05
mkdir -p $O
for a in 0 32 0 32; do
  PNP_LIB_PATH=pnp-pds_amd/lib_prof/libpnppds.so timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --converge-run 0 --ablate-k2 $a >> $O/k2ab_fp32_fp64.jsonl 2>> $O/k2ab.err || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_graph.py tests/test_gpu_iter.py tests/test_gpu_configs.py -v -s --timeout 300 --timeout-method thread > $O/pytest_run3.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
export PNP_BENCH_REHEARSAL=1 MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --batch 64 > $O/rehearse_n2.json 2> $O/rehearse_n2.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --steps 4 --warmup 1 --batch 64 > $O/rehearse_n2_self.json 2> $O/rehearse_n2_self.err || exit 1
exit $rc
