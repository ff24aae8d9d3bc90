# PMC passes of the B = 1 stack (cfg2): LDS bank conflicts, MFMA busy, waits
set -e
mkdir -p gpurun_out/r04/pmc_stack
export TMPDIR=/tmp
P="python3 bench.py --config cfg2 --steps 20 --warmup 2 --no-cpu-baseline --profile 0"
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/r04/pmc_stack -o a --output-format csv -- $P > gpurun_out/r04/pmc_stack/a.log 2>&1
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD -d gpurun_out/r04/pmc_stack -o b --output-format csv -- $P > gpurun_out/r04/pmc_stack/b.log 2>&1
python3 tools/pmc_summary.py $(find gpurun_out/r04/pmc_stack -name "*_counter_collection.csv") > gpurun_out/r04/pmc_stack/summary.txt
grep -A20 "conv_stack16x2" gpurun_out/r04/pmc_stack/summary.txt | head -24
