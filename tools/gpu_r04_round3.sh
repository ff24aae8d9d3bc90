set -e
mkdir -p gpurun_out/r04
bash tools/gpu_r04_ab_wpe.sh
timeout -k 10 1000 python -u -m pytest tests/ -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r04/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04/pytest_gpu.log
for c in cfg2 cfg1; do
timeout -k 10 120 python3 -u bench.py --config $c --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c latency', d['ms_per_step'])"
done
