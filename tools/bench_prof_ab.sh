# bench timed region with and without the per-kernel HIP-event scopes
set -e
for p in 0 1 0 1; do timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --profile $p 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('profile', $p, d['value'], d['ms_per_step'], round(sum(d.get('kernel_ms',{}).values()),3))"; done
