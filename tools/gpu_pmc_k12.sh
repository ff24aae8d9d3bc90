# PMC passes over the metric bench for the blur passes (K1 / K2): issue, waits, instruction mix, traffic
D=${1:-gpurun_out/pmck12}; mkdir -p $D; export TMPDIR=/tmp
P="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile 0"
R="--kernel-include-regex k1_blur|k2_blur"
timeout -s KILL 240 rocprofv3 $R --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $D -o a --output-format csv -- $P > $D/a.log 2>&1 || exit 11
timeout -s KILL 240 rocprofv3 $R --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM -d $D -o b --output-format csv -- $P > $D/b.log 2>&1 || exit 12
timeout -s KILL 240 rocprofv3 $R --pmc FETCH_SIZE TA_BUSY_avr TA_TA_BUSY_sum -d $D -o c --output-format csv -- $P > $D/c.log 2>&1 || exit 13
timeout -s KILL 240 rocprofv3 $R --pmc WRITE_SIZE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MUL_F64 -d $D -o d --output-format csv -- $P > $D/d.log 2>&1 || echo "pass d failed (optional)"
python3 tools/pmc_summary.py $(find $D -name "*_counter_collection.csv") > $D/summary.txt
cat $D/summary.txt
