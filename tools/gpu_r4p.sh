# configs[1] recurrence (fp32, B 1024, H 512): per-step kernel variants, then a kernel trace
# (per-launch duration against the wall time per step)
mkdir -p gpurun_out
for rows in 128 256; do
  TT_GRU_FWD_STEP_ROWS=$rows timeout -k 10 200 python tools/bench_gru.py --dtype fp32 --B 1024 --H 512 --T 64 --iters 5 --variants "step:0,step:0" --bwd-variants "S:0:2,S:0:1,64:0:2,64:0:1" > gpurun_out/r4p_rows$rows.txt 2>&1 || exit 1
  echo "== fwd rows $rows"; grep -v amdgpu gpurun_out/r4p_rows$rows.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4p_prof -o p -- python $GRAFT_REPO_ROOT/tools/bench_gru.py --dtype fp32 --B 1024 --H 512 --T 64 --iters 3 --variants "step:0" --bwd-variants "S:0:2" > $GRAFT_REPO_ROOT/gpurun_out/r4p_prof.log 2>&1 || exit 1
echo prof ok
