# Buffer-resource operand DMAs in the 8-phase GEMM (option gemm_buf): parity, GEMM A/B, step A/B
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_buf.py tests/test_gpu_kernels.py tests/test_gpu_bench_path.py tests/test_gpu_hardneg.py tests/test_gpu_gru_persistent.py tests/test_gpu_model.py > gpurun_out/r4g_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r4g_pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm.py --shapes square8k,input_proj_l1,dgrad_l1,wgrad_hh,wgrad_ih1,c4_proj_l1,c4_dgrad_l1 --iters 10 --rounds 2 --variants "gemm_buf=0;gemm_buf=1" > gpurun_out/r4g_gemm.txt 2>&1 || exit 1
cat gpurun_out/r4g_gemm.txt | grep -v amdgpu.ids
for v in 1 0 1 0; do
  TT_GEMM_BUF=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4g_bench_$v.json 2>> gpurun_out/r4g_bench.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r4g_bench_$v.json')); k=d['kernel_ms_per_step']; print('buf=$v', d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
done
