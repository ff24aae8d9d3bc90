D=gpurun_out/pmck; mkdir -p $D; export TMPDIR=/tmp
P="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile 0"
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $D -o a --output-format csv -- $P > $D/a.log 2>&1 || exit 11
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $D -o b --output-format csv -- $P > $D/b.log 2>&1 || exit 12
echo pmc-ok
