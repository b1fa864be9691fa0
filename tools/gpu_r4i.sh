# gru_bwd_rows carry through the accumulator image (TT_BWD_CREG): parity, kernel A/B, step
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_bench_path.py tests/test_gpu_golden.py tests/test_gpu_gru_persistent.py tests/test_gpu_gemm_buf.py > gpurun_out/r4i_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r4i_pytest.txt
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libtt_hip.so libtt_hip_exp.so; do
  echo "== $lib"; TT_HIP_LIB=$GRAFT_REPO_ROOT/two_towers_amd/lib/$lib timeout -k 10 200 python tools/bench_gru.py --variants "" --bwd-variants P:0:2:14,P:0:2:0 --iters 5 || exit 1
done; done > gpurun_out/r4i_bwd_ab.txt 2>&1
grep -v amdgpu gpurun_out/r4i_bwd_ab.txt
for lib in libtt_hip.so libtt_hip_exp.so libtt_hip.so; do
  TT_HIP_LIB=$GRAFT_REPO_ROOT/two_towers_amd/lib/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4i_bench.json 2>> gpurun_out/r4i_bench.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r4i_bench.json')); k=d['kernel_ms_per_step']; print('$lib', d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
done
cp gpurun_out/r4i_bench.json gpurun_out/r4i_bench_final.json
