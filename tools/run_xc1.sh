set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gru_persistent.py -k "column_split or bench_grid" > gpurun_out/xc1_pytest.log 2>&1
rc=$?
tail -25 gpurun_out/xc1_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_gru.py --variants seq:0,xc:0,xc:0 --bwd-variants "" --iters 5 > gpurun_out/xc1_bench.log 2>&1
rc=$?; cat gpurun_out/xc1_bench.log | tail; exit $rc
