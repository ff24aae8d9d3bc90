# conv_body_v3 ablation, kernel-trace timings only (no PMC), B=256 structured inputs
D=${1:-gpurun_out/ablkt}; mkdir -p $D; export TMPDIR=/tmp
for ab in 0 1 2 3 4 5 6; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D -o ab$ab --output-format csv -- python3 tools/prof_denoise.py --batch 256 --reps 3 --variant 0 --ablate $ab > $D/ab$ab.log 2>&1 || exit 31
done
echo ablkt-ok
