set -e
BARGS0="--steps 10" KFILT=conv bash tools/gpu_ab.sh
BARGS0="--steps 4 --warmup 1" KFILT=k_ CFGS=cfg4 bash tools/gpu_ab.sh
CFGS="cfg2" bash tools/gpu_ab_lat.sh
