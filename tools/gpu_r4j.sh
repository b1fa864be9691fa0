# non-temporal once-read loads in the backward epilogue (nt1: S, nt3: S + dy + h) vs default; then the bookkeeping (r4e)
mkdir -p gpurun_out
for rep in 1 2; do for lib in libtt_hip.so libtt_hip_nt1.so libtt_hip_nt3.so; do
  echo "== $lib"; TT_HIP_LIB=$GRAFT_REPO_ROOT/two_towers_amd/lib/$lib timeout -k 10 200 python tools/bench_gru.py --variants "" --bwd-variants P:0:2:14 --iters 5 || exit 1
done; done > gpurun_out/r4j_bwd_nt.txt 2>&1
grep -v amdgpu gpurun_out/r4j_bwd_nt.txt
bash tools/gpu_r4e.sh
