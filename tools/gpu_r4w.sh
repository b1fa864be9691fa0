# 128x128 GEMM tiles with the 4-stage ring (option gemm_ring) at one workgroup per CU: parity, step A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_golden.py tests/test_gpu_model.py tests/test_gpu_gemm_buf.py > gpurun_out/r4w_pytest.txt 2>&1; rc=$?; tail -2 gpurun_out/r4w_pytest.txt
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in 4 2; do
  TT_GEMM_RING=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4w_c2_ring${v}_$rep.json 2>> gpurun_out/r4w_bench.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r4w_c2_ring${v}_$rep.json')); print('c2 gemm_ring=$v', d['value'], d['ms_per_step'])
"
done; done
for v in 4 2; do
  TT_GEMM_RING=$v timeout -k 10 300 python bench.py --batch 1024 --dtype fp32 --loss infonce --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4w_c1_ring$v.json 2>> gpurun_out/r4w_bench.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r4w_c1_ring$v.json')); print('c1 gemm_ring=$v', d['value'], d['ms_per_step'])
"
done
cd /tmp && export TMPDIR=/tmp
for v in 4 2; do
TT_GEMM_RING=$v TT_GRU_XC_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4w_prof$v -o p -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r4w_prof$v.log 2>&1 || exit 1
done
echo prof ok
