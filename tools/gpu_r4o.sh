# dW_hh shifted operand with per-K-tile resource bases (masked lanes one K-tile ahead):
# parity, then configs[2] with buffer DMAs on / off, then the final-build validation
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_buf.py > gpurun_out/r4o_pytest.txt 2>&1; rc=$?; tail -2 gpurun_out/r4o_pytest.txt
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  TT_GEMM_BUF=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4o_bench_buf$v.json 2>> gpurun_out/r4o_bench.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r4o_bench_buf$v.json')); k=d['kernel_ms_per_step']; print('c2 buf=$v', d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
done
bash tools/gpu_r4n.sh
