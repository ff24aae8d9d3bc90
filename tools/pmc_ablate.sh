# effective clock / MFMA busy of conv_body per ablation mode (profiling only)
mkdir -p gpurun_out/pmcab; export TMPDIR=/tmp
for ab in 0 3 4 6; do
  PNPPDS_ABLATE=$ab timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmcab -o ab$ab --output-format csv -- python3 tools/prof_denoise.py --batch 64 --reps 2 --variant 1 > gpurun_out/pmcab/ab$ab.log 2>&1 || exit 31
done
echo pmcab-ok
