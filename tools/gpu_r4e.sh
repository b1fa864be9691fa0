# Round-4 final-build bookkeeping: bench line + rocprof kernel stats, PMC traffic passes,
# the CPU baseline at the metric's batch (B 8192, 1 warm-up + 2 timed steps)
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4e_bench.json 2> gpurun_out/r4e_bench.err || exit 1
cat gpurun_out/r4e_bench.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4e_prof -o p -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r4e_prof.log 2>&1 ) || exit 1
timeout -k 10 900 bash tools/pmc_bench.sh r4e || exit 1
timeout -k 10 900 python bench.py --cpu-only --cpu-batch 8192 --cpu-steps 2 --cpu-warmup 1 > gpurun_out/r4e_cpu_b8192.json 2> gpurun_out/r4e_cpu_b8192.err || exit 1
cat gpurun_out/r4e_cpu_b8192.json
