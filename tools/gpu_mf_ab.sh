# MFMA blur A/B: bench kernel times for the abl_libs/*.so variants, plus the VALU stencils (BLUR_MFMA=0) on the product lib
set -e
mkdir -p gpurun_out
CFGS=metric KFILT=zz timeout -k 10 300 bash tools/gpu_ab.sh
timeout -k 10 120 python -u bench.py --steps 10 --no-cpu-baseline --blur-mfma 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print('valu', d['value'], {a: round(b, 4) for a, b in k.items()})"
