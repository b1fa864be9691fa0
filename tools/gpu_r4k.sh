# CPU baseline at the metric's batch; then rocprofv3 kernel stats of the step with the
# column-split forward launched plainly (gru_xc_coop 0) and cooperatively (default): the
# round-4 bench crashed in process teardown under rocprofv3 (after its output was written)
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --cpu-only --cpu-batch 8192 --cpu-steps 2 --cpu-warmup 1 > gpurun_out/r4k_cpu_b8192.json 2> gpurun_out/r4k_cpu_b8192.err || exit 1
cat gpurun_out/r4k_cpu_b8192.json
cd /tmp && export TMPDIR=/tmp
TT_GRU_XC_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4k_prof_nocoop -o p -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r4k_prof_nocoop.log 2>&1 || { echo "nocoop rc=$?"; exit 1; }
echo nocoop ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4k_prof -o p -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r4k_prof.log 2>&1 || { echo "coop rc=$?"; exit 1; }
echo coop ok
