# PMC passes over the bench command for the prox/operator kernels (profiling only)
D=${1:-gpurun_out/pmcprox}; mkdir -p $D; export TMPDIR=/tmp
P="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile 0"
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $D -o a --output-format csv -- $P > $D/a.log 2>&1 || exit 11
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $D -o b --output-format csv -- $P > $D/b.log 2>&1 || exit 12
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $D -o c --output-format csv -- $P > $D/c.log 2>&1 || exit 13
timeout -k 10 240 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $D -o d --output-format csv -- $P > $D/d.log 2>&1 || exit 14
timeout -k 10 240 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES SQ_INSTS_SMEM SQ_IFETCH SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $D -o e --output-format csv -- $P > $D/e.log 2>&1 || echo "pass e failed (optional)"
echo pmc-ok
