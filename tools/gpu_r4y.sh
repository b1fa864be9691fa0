# dW_hh's time-shifted operand: 32-bit / power-of-two time advance per K-tile (libtt_hip) vs the
# 64-bit modulo (libtt_hip_prev): parity of the shifted GEMM, then configs[2] A/B on one box
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_buf.py tests/test_gpu_kernels.py > gpurun_out/r4y_pytest.txt 2>&1; rc=$?; tail -2 gpurun_out/r4y_pytest.txt
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for lib in libtt_hip.so libtt_hip_prev.so; do
  TT_HIP_LIB=$GRAFT_REPO_ROOT/two_towers_amd/lib/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4y_$lib.$rep.json 2>> gpurun_out/r4y_bench.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r4y_$lib.$rep.json')); k=d['kernel_ms_per_step']; print('$lib', d['value'], d['ms_per_step'], 'wgrad_hh', k['wgrad_hh']['ms_per_step'])
"
done; done
