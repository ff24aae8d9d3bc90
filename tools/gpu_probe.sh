# long-trajectory |dPSNR| probe (no asserts): cases..., last arg = comma-separated precisions
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/long_parity_probe.py "$@" > gpurun_out/probe.log 2>&1 || { tail -20 gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
