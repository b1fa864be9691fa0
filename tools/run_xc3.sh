set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_gru_persistent.py -k "column_split_forward or bench_grid" > gpurun_out/xc3_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/xc3_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_gru.py --variants seq:0,xco:0,xc:0,xcs:0,xco:0,xc:0 --bwd-variants "" --iters 5 > gpurun_out/xc3_bench.log 2>&1
rc=$?; cat gpurun_out/xc3_bench.log | grep variant; exit $rc
