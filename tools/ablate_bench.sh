# conv_body_v3 ablation inside the bench loop (profiling only; the solver output is wrong when ablated)
D=${1:-gpurun_out/ablb}; mkdir -p $D
for ab in 0 3 4 6; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --variant 0 --ablate $ab > $D/ab$ab.json 2> $D/ab$ab.log || exit 31
done
echo ablb-ok
