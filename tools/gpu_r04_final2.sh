# round-4 close, the tree as committed: the whole GPU suite, smoke(), the default bench line, cfg1 / cfg2 latency
set -e
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_close.log 2>&1 || { tail -30 gpurun_out/r04/pytest_close.log; exit 1; }
tail -2 gpurun_out/r04/pytest_close.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 600 python -u bench.py > gpurun_out/r04/bench_close.json 2> gpurun_out/r04/bench_close.err
cat gpurun_out/r04/bench_close.json
for c in cfg2 cfg1; do
timeout -k 10 120 python3 -u bench.py --config $c --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c latency', d['ms_per_step'])"
done
