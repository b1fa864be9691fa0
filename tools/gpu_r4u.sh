# fp32 per-step forward with the epilogue loads issued before the product: parity, diag split, configs[1]
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_kernels.py tests/test_gpu_model.py > gpurun_out/r4u_pytest.txt 2>&1; rc=$?; tail -2 gpurun_out/r4u_pytest.txt
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  TT_HIP_LIB=$GRAFT_REPO_ROOT/two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 200 python tools/bench_gru.py --dtype fp32 --B 1024 --H 512 --T 64 --iters 5 --variants "step:0,step:8,step:16" --bwd-variants "" || exit 1
  for ring in 4 2; do echo "== ring $ring"; TT_GRU_STEP_RING=$ring timeout -k 10 200 python tools/bench_gru.py --dtype fp32 --B 1024 --H 512 --T 64 --iters 5 --variants "step:0" --bwd-variants "" || exit 1; done
done > gpurun_out/r4u_fwd.txt 2>&1
grep -v amdgpu gpurun_out/r4u_fwd.txt
timeout -k 10 300 python bench.py --batch 1024 --dtype fp32 --loss infonce --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4u_bench_c1.json 2>> gpurun_out/r4u_bench.err || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/r4u_bench_c1.json')); k=d['kernel_ms_per_step']; print('c1', d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
