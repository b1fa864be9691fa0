# per-step GRU product ring (option gru_step_ring): parity, fp32 recurrence A/B, configs[1] lines
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_gru_persistent.py > gpurun_out/r4r_pytest.txt 2>&1; rc=$?; tail -2 gpurun_out/r4r_pytest.txt
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for ring in 2 3 4; do
  echo "== ring $ring"; TT_GRU_STEP_RING=$ring timeout -k 10 200 python tools/bench_gru.py --dtype fp32 --B 1024 --H 512 --T 64 --iters 5 --variants "step:0" --bwd-variants "64:0:2,64:0:1" || exit 1
done; done > gpurun_out/r4r_ring.txt 2>&1
grep -v amdgpu gpurun_out/r4r_ring.txt
for v in 4:2 2:2 4:1; do ring=${v%:*}; strm=${v#*:}
  TT_GRU_BWD_STREAMS=$strm TT_GRU_STEP_RING=$ring timeout -k 10 300 python bench.py --batch 1024 --dtype fp32 --loss infonce --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4r_bench_c1_ring${ring}_s$strm.json 2>> gpurun_out/r4r_bench.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r4r_bench_c1_ring${ring}_s$strm.json')); k=d['kernel_ms_per_step']; print('c1 ring=$ring streams=$strm', d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
done
