# graph replay: parity tests, then B = 1 latency with / without graphs (HIP-event scopes off)
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_iter.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/graph_pytest.log 2>&1 || { tail -40 gpurun_out/graph_pytest.log; exit 1; }
tail -1 gpurun_out/graph_pytest.log
for c in cfg1 cfg2; do for G in 1 2; do
timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 200 --warmup 10 --profile 0 --graph $G > gpurun_out/graph_${c}_$G.json 2>gpurun_out/graph_${c}_$G.err
python -c "import json; d=json.load(open('gpurun_out/graph_${c}_$G.json')); print('$c graph$G', d['value'], d['ms_per_step'])"
done; done
