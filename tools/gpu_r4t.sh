# fp32 per-step recurrences at configs[1], diagnostic build (timing only): forward without the
# product (8) / the epilogue (16) / both; backward without the product (1) / epilogue loads
# and stores (6)
mkdir -p gpurun_out
for rep in 1 2; do
  TT_HIP_LIB=$GRAFT_REPO_ROOT/two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 200 python tools/bench_gru.py --dtype fp32 --B 1024 --H 512 --T 64 --iters 5 --variants "step:0,step:8,step:16,step:24" --bwd-variants "64:0:2,64:1:2,64:6:2,64:7:2" || exit 1
done > gpurun_out/r4t_diag.txt 2>&1
grep -v amdgpu gpurun_out/r4t_diag.txt
