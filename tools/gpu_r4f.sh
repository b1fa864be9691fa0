# Loop8 main-loop diagnostics: the product library vs no in-loop DMA (l8d1) vs DMA without
# per-K-tile address arithmetic (l8d2); timing only for the diagnostic builds
mkdir -p gpurun_out
for rep in 1 2; do for lib in libtt_hip.so libtt_hip_l8d1.so libtt_hip_l8d2.so; do
  echo "== $lib"; TT_HIP_LIB=$GRAFT_REPO_ROOT/two_towers_amd/lib/$lib timeout -k 10 200 python tools/bench_gemm.py --shapes square8k,input_proj_l1,dgrad_l1,wgrad_hh,wgrad_ih1 --iters 10 || exit 1
done; done > gpurun_out/r4f_gemm_diag.txt 2>&1
cat gpurun_out/r4f_gemm_diag.txt
