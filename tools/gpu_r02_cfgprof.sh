# cfg5 bench line (HBM-sized denoiser passes) and kernel traces of cfg3 / cfg5 (l1_select's kernels at 256^2 and 1024^2).
set -e
mkdir -p gpurun_out/r02 gpurun_out/prof_cfg
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config cfg5 --steps 3 --warmup 1 > gpurun_out/r02/bench_cfg5.json 2> gpurun_out/r02/bench_cfg5.err
python -c "import json; d=json.load(open('gpurun_out/r02/bench_cfg5.json')); print('cfg5', d['value'], d['ms_per_step'], d['roofline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg -o trace_cfg3 --output-format csv -- python3 bench.py --config cfg3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_cfg/cfg3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg -o trace_cfg5 --output-format csv -- python3 bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_cfg/cfg5.log 2>&1
find gpurun_out/prof_cfg -name "*kernel_stats.csv"
