# Round-3 measurements, part 1: the default bench with its rocprofv3 kernel trace and PMC passes
# (outputs under gpurun_out/r03/bench/).  Part 2 (the per-config lines): tools/gpu_r03_profile.sh SKIP_BENCH=1.
set -e
mkdir -p gpurun_out/r03/bench
export TMPDIR=/tmp
bash tools/profile_bench.sh gpurun_out/r03/bench
F=$(find gpurun_out/r03/bench -name "pmc_fetch_counter_collection.csv" | head -1)
W=$(find gpurun_out/r03/bench -name "pmc_write_counter_collection.csv" | head -1)
python3 tools/traffic_from_pmc.py $F $W --out gpurun_out/r03/bench/traffic.json > /dev/null
python3 tools/pmc_summary.py $(find gpurun_out/r03/bench -name "pmc_*_counter_collection.csv") > gpurun_out/r03/bench/pmc_summary.txt
python3 -c "import json; d=json.load(open('gpurun_out/r03/bench/bench.json')); print('metric', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernel_ms'], d.get('prox_hbm'))"
