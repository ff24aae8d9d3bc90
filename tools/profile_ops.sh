# Bench lines + kernel trace of the pointwise-operator paths (Id, random_sampling), profiling only.
#   bash tools/profile_ops.sh <outdir>
D=${1:-gpurun_out/prof_ops}
mkdir -p $D; export TMPDIR=/tmp
for op in Id random_sampling; do
  timeout -k 10 300 python3 bench.py --op $op --no-cpu-baseline > $D/bench_$op.json 2> $D/bench_$op.log || exit 20
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o trace_rs --output-format csv -- python3 bench.py --op random_sampling --steps 10 --warmup 2 --no-cpu-baseline > $D/trace_rs.log 2>&1 || exit 21
echo profile-ok $D
