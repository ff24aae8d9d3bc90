# conv_body_v3 ablation (profiling only): kernel time / clock / MFMA busy per mode, B=256
D=${1:-gpurun_out/abl}; mkdir -p $D; export TMPDIR=/tmp
for ab in 0 1 2 3 4 5; do
  timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY -d $D -o ab$ab --output-format csv -- python3 tools/prof_denoise.py --batch 256 --reps 2 --variant 0 --ablate $ab > $D/ab$ab.log 2>&1 || exit 31
done
echo abl-ok
