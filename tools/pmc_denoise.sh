mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
P="python3 tools/prof_denoise.py --batch 64 --reps 2"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc -o passA --output-format csv -- $P > gpurun_out/pmc/a.log 2>&1 || exit 11
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d gpurun_out/pmc -o passB --output-format csv -- $P > gpurun_out/pmc/b.log 2>&1 || exit 12
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o passC --output-format csv -- $P > gpurun_out/pmc/c.log 2>&1 || exit 13
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc -o passD --output-format csv -- $P > gpurun_out/pmc/d.log 2>&1 || exit 14
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc -o trace --output-format csv -- $P > gpurun_out/pmc/t.log 2>&1 || exit 15
echo pmc-ok
