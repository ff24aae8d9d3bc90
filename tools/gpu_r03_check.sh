# round 3: full GPU suite + cfg1 / cfg4 bench lines (cfg1 with its CPU baseline and PSNR delta vs the oracle)
set -e
mkdir -p gpurun_out/r03
bash tools/gpu_tests.sh
timeout -k 10 300 python -u bench.py --config cfg1 --cpu-budget 10 > gpurun_out/r03/bench_cfg1.json 2> gpurun_out/r03/bench_cfg1.err
timeout -k 10 300 python -u bench.py --config cfg4 --no-cpu-baseline > gpurun_out/r03/bench_cfg4.json 2> gpurun_out/r03/bench_cfg4.err
python -c "
import json
for f in ('bench_cfg1','bench_cfg4'):
    d=json.loads(open('gpurun_out/r03/'+f+'.json').read())
    print(f, d['value'], d['ms_per_step'], d['config']['precision'], d.get('psnr_delta_db_vs_oracle'))
"
