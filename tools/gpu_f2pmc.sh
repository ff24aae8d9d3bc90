# SQ / LDS counters of the one-layer and the fused two-layer body kernel (profiling only)
set -e
for L in 1 2; do
bash tools/pmc_body.sh 256 gpurun_out/f2pmc$L --body-layers $L
python3 tools/pmc_summary.py gpurun_out/f2pmc$L/passA_counter_collection.csv gpurun_out/f2pmc$L/passB_counter_collection.csv --kernel conv_body > gpurun_out/f2pmc$L/summary.txt
cat gpurun_out/f2pmc$L/summary.txt
done
