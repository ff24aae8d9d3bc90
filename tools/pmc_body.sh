# PMC passes for the denoiser (profiling only): bash tools/pmc_body.sh <batch> <outdir> [extra prof_denoise args]
B=${1:-64}; D=${2:-gpurun_out/pmc_den}; shift 2
mkdir -p $D; export TMPDIR=/tmp
P="python3 tools/prof_denoise.py --batch $B --reps 2 $*"
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $D -o passA --output-format csv -- $P > $D/a.log 2>&1 || exit 11
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $D -o passB --output-format csv -- $P > $D/b.log 2>&1 || exit 12
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $D -o passC --output-format csv -- $P > $D/c.log 2>&1 || exit 13
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $D -o passD --output-format csv -- $P > $D/d.log 2>&1 || exit 14
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D -o trace --output-format csv -- $P > $D/t.log 2>&1 || exit 15
echo pmc-ok $D
