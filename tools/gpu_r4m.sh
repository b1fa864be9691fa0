# fp32 buffer DMAs and the column-group tile walk (parity), GEMM A/B, backward epilogue batch NB 4, forward G loads non-temporal, configs[1] line
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_buf.py tests/test_gpu_kernels.py tests/test_gpu_golden.py tests/test_gpu_model.py tests/test_gpu_bench_path.py > gpurun_out/r4m_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r4m_pytest.txt
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libtt_hip.so libtt_hip_s0.so libtt_hip_nb4.so; do
  echo "== $lib"; TT_HIP_LIB=$GRAFT_REPO_ROOT/two_towers_amd/lib/$lib timeout -k 10 200 python tools/bench_gru.py --variants "" --bwd-variants P:0:2:14,P:0:2:0,P:0:2:7 --iters 5 || exit 1
done; done > gpurun_out/r4m_bwd.txt 2>&1
grep -v amdgpu gpurun_out/r4m_bwd.txt
timeout -k 10 300 python tools/bench_gemm.py --shapes input_proj_l1,c4_proj_l1 --iters 10 --rounds 2 --variants "gemm_order=0;gemm_order=1" > gpurun_out/r4m_order.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r4m_order.txt
for rep in 1 2; do for lib in libtt_hip.so libtt_hip_xg2.so; do
  echo "== $lib"; TT_HIP_LIB=$GRAFT_REPO_ROOT/two_towers_amd/lib/$lib timeout -k 10 200 python tools/bench_gru.py --variants "xc:0,xc:0" --bwd-variants "" --iters 5 || exit 1
done; done > gpurun_out/r4m_fwd.txt 2>&1
grep -v amdgpu gpurun_out/r4m_fwd.txt
for v in 1 0; do
  TT_GEMM_BUF=$v timeout -k 10 300 python bench.py --batch 1024 --dtype fp32 --loss infonce --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4m_bench_c1_$v.json 2>> gpurun_out/r4m_bench.err || exit 1
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/r4m_bench_c1_$v.json')); k=d['kernel_ms_per_step']; print('c1 buf=$v', d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4m_bench.json 2>> gpurun_out/r4m_bench.err || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/r4m_bench.json')); k=d['kernel_ms_per_step']; print('c2', d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
