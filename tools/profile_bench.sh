# Round profile of the benchmark command (kernel trace + HBM / SQ counters), profiling only.
#   bash tools/profile_bench.sh <outdir> [extra bench args]
D=${1:-gpurun_out/prof}; shift
mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py "$@" > $D/bench.json 2> $D/bench.log || exit 20
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o trace --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --converge-run 0 "$@" > $D/trace.log 2>&1 || exit 21
P="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --converge-run 0 --profile 0 $*"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $D -o pmc_fetch --output-format csv -- $P > $D/pmc_fetch.log 2>&1 || exit 22
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $D -o pmc_write --output-format csv -- $P > $D/pmc_write.log 2>&1 || exit 23
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU -d $D -o pmc_sq --output-format csv -- $P > $D/pmc_sq.log 2>&1 || exit 24
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD -d $D -o pmc_lds --output-format csv -- $P > $D/pmc_lds.log 2>&1 || exit 25
echo profile-ok $D
