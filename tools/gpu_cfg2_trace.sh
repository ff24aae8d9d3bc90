# rocprofv3 kernel trace of the B = 1 cfg2 latency run (profiling only): per-kernel durations without event scopes
set -e
mkdir -p gpurun_out/cfg2tr; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg2tr -o tr --output-format csv -- python3 bench.py --config cfg2 --profile 0 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/cfg2tr/bench.log 2>&1
F=$(find gpurun_out/cfg2tr -name "tr_kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$F')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:16]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,2), 'us')
"
