mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hardneg.py tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_path.py > gpurun_out/r4c_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r4c_pytest.txt
[ $rc -eq 0 ] || exit $rc
bash tools/ab_scan.sh r4c libtt_hip.so libtt_hip_exp.so > gpurun_out/r4c_scan.txt 2>&1 || exit 1
for d in gpurun_out/abscan_r4c/*_1 gpurun_out/abscan_r4c/*_2; do echo "== $d"; python3 tools/kstats.py $(ls $d/*kernel_trace.csv) hn_scan; done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err || exit 1
TT_GEMM_BRES=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4c_bench_nobres.json 2>> gpurun_out/r4c_bench.err || exit 1
timeout -k 10 400 python bench.py --hidden 512 --seq 128 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4c_bench_c4.json 2>> gpurun_out/r4c_bench.err || exit 1
TT_GRU_BWD_PERSIST=0 timeout -k 10 400 python bench.py --hidden 512 --seq 128 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4c_bench_c4_old.json 2>> gpurun_out/r4c_bench.err || exit 1
python3 -c "
import json
for f in ('r4c_bench','r4c_bench_nobres','r4c_bench_c4','r4c_bench_c4_old'):
    d=json.load(open('gpurun_out/'+f+'.json')); k=d['kernel_ms_per_step']; print(f, d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
for v in "" "TT_GRU_BWD_ROWS=64" "TT_GRU_BWD_STREAMS=1"; do
  env $v timeout -k 10 300 python bench.py --batch 1024 --dtype fp32 --loss infonce --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4c_bench_c1.json 2>> gpurun_out/r4c_bench.err || exit 1
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/r4c_bench_c1.json')); k=d['kernel_ms_per_step']; print('c1 $v', d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
done
