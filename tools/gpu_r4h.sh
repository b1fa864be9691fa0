# r4d's diagnostics (its pytest ran in r4d/r4g): backward skew and phase diagnostics,
# configs[1] variants, hn_scan block maps and query-prologue A/B
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4h_smoke.txt 2>&1 || exit 1
cat gpurun_out/r4h_smoke.txt | grep smoke
bash tools/ab_scan.sh r4h libtt_hip.so libtt_hip_exp.so > gpurun_out/r4h_scan.txt 2>&1 || exit 1
cat gpurun_out/r4h_scan.txt
TT_HIP_LIB=two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 300 python tools/bench_gru.py --variants "" --bwd-variants P:0:2:14,P:1:2:14,P:2:2:14,P:4:2:14,P:6:2:14,P:7:2:14,P:0:2:0,P:1:2:0,P:6:2:0 --iters 5 > gpurun_out/r4h_bwd_diag.txt 2>&1 || exit 1
cat gpurun_out/r4h_bwd_diag.txt
for rep in 1 2; do
timeout -k 10 200 python tools/bench_score.py --ops hardneg --iters 50 --hn-shapes 8192x8192x256,8192x65536x256 --variants "map1=hn_map=1;map2=hn_map=2" >> gpurun_out/r4h_hnmap.txt 2>&1 || exit 1
done
cat gpurun_out/r4h_hnmap.txt
# gru_bwd_rows product DMAs through buffer resources (libtt_hip) vs per-lane pointers (libtt_hip_exp: TT_BWD_BUF=0)
for rep in 1 2; do for lib in libtt_hip.so libtt_hip_exp.so; do
  echo "== $lib"; TT_HIP_LIB=$GRAFT_REPO_ROOT/two_towers_amd/lib/$lib timeout -k 10 200 python tools/bench_gru.py --variants "" --bwd-variants P:0:2:14 --iters 5 || exit 1
done; done > gpurun_out/r4h_bwd_buf.txt 2>&1
cat gpurun_out/r4h_bwd_buf.txt | grep -v amdgpu.ids
