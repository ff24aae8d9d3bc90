export TMPDIR=/tmp
for V in ${PMCV:-0 3}; do D=gpurun_out/pmcv$V; mkdir -p $D
P="python3 tools/prof_denoise.py --batch 64 --reps 2 --variant $V"
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $D -o passA --output-format csv -- $P > $D/a.log 2>&1 || exit 11
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $D -o passB --output-format csv -- $P > $D/b.log 2>&1 || exit 12
done; echo ok
