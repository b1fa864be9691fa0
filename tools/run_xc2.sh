set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_gru_persistent.py -k "column_split or bench_grid" > gpurun_out/xc2_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/xc2_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_gru.py --variants seq:0,xc:0,xc:0 --bwd-variants "" --iters 5 > gpurun_out/xc2_bench.log 2>&1
rc=$?; cat gpurun_out/xc2_bench.log | grep variant; [ $rc -ne 0 ] && exit $rc
TT_HIP_LIB=two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 200 python -u tools/diag_xc.py 0 1 2 4 6 7 > gpurun_out/xc2_diag.log 2>&1
rc=$?; cat gpurun_out/xc2_diag.log | grep dbg; exit $rc
