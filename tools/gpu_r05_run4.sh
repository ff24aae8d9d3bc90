#!/bin/bash
# r05 run 4: K2 without x_true loads (ABL 64) vs the product, and PMC passes of the split-activation
# body kernels (fp16a2, fp16x3) on the denoiser alone (B = 64 RGB 256^2)
set -o pipefail
O=gpurun_out/r05
mkdir -p $O; export TMPDIR=/tmp
for a in 0 64 0 64; do
  PNP_LIB_PATH=pnp-pds_amd/lib_prof/libpnppds.so timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --converge-run 0 --ablate-k2 $a >> $O/k2ab_xtrue.jsonl 2>> $O/k2ab_xtrue.err || exit 1
done
for p in fp16a2 fp16x3; do
  D=$O/pmc_$p; mkdir -p $D
  P="python3 tools/prof_denoise.py --batch 64 --reps 2 --precision $p"
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU -d $D -o sq --output-format csv -- $P > $D/sq.log 2>&1 || exit 11
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD -d $D -o lds --output-format csv -- $P > $D/lds.log 2>&1 || exit 12
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $D -o fetch --output-format csv -- $P > $D/fetch.log 2>&1 || exit 13
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $D -o write --output-format csv -- $P > $D/write.log 2>&1 || exit 14
done
echo ok
