# SQ counter pass over the cfg4 bench (split-fp16 body): MFMA busy, clock, VALU of conv_s3
set -e
D=gpurun_out/pmc_cfg4; mkdir -p $D; export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU -d $D -o pmc_sq --output-format csv -- python3 bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline --profile 0 > $D/log 2>&1
python3 tools/pmc_summary.py $(find $D -name "pmc_sq_counter_collection.csv") > $D/pmc_summary.txt
grep -A 14 "conv_s3_kernel" $D/pmc_summary.txt | head -34
