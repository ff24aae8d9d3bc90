# One SQ counter pass over the metric bench (profiling only): VALU / MFMA / clock of each kernel.
#   bash tools/gpu_pmc_sq.sh <outdir> [extra bench args]
D=${1:-gpurun_out/pmc_sq}; shift
mkdir -p $D; export TMPDIR=/tmp
P="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile 0 $*"
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU -d $D -o pmc_sq --output-format csv -- $P > $D/pmc_sq.log 2>&1 || exit 24
python3 tools/pmc_summary.py $(find $D -name "pmc_sq_counter_collection.csv") > $D/pmc_summary.txt
grep -A 12 "conv_body_x8" $D/pmc_summary.txt
