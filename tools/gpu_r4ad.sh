# configs[1] (fp32, B 1024) kernel statistics on the final build
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4ad_prof -o p -- python $GRAFT_REPO_ROOT/bench.py --batch 1024 --dtype fp32 --loss infonce --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r4ad_prof.log 2>&1 || exit 1
echo prof ok
