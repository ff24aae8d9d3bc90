set -e
for spec in "metric fp16w2" "cfg4 fp32" "cfg4 fp16w2" "cfg4 fp16"; do set -- $spec
timeout -k 10 300 python -u bench.py --config $1 --precision $2 --no-cpu-baseline --steps 10 > gpurun_out/w2b_$1_$2.json 2>gpurun_out/w2b_$1_$2.err
python -c "import json; d=json.load(open('gpurun_out/w2b_$1_$2.json')); print('$1 $2', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('roofline',{}).get('frac'))"
done
