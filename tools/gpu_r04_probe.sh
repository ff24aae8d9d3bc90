# round 4: FETCH_SIZE / WRITE_SIZE calibration probe; cooperative vs plain stack launches at B = 1
set -e
mkdir -p gpurun_out/r04/probe
export TMPDIR=/tmp
timeout -k 10 60 tools/probes/fetch_probe > gpurun_out/r04/probe/fetch_probe.txt
cat gpurun_out/r04/probe/fetch_probe.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04/probe -o fetch -- tools/probes/fetch_probe > gpurun_out/r04/probe/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r04/probe -o write -- tools/probes/fetch_probe > gpurun_out/r04/probe/write.log 2>&1
for r in 1 2; do for L in coop plain; do for c in cfg2 cfg1; do
PNP_LIB_PATH=$PWD/abl_libs/$L.so timeout -k 10 200 python -u bench.py --config $c --profile 0 --steps 300 --warmup 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L $c', d['ms_per_step'], d['value'])"
done; done; done
