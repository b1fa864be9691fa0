set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gru_persistent.py -k "column_split_forward or h1024 or bench_grid" > gpurun_out/xk1_pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|identical" gpurun_out/xk1_pytest.log | grep -E "FAIL|h1024|Y0" | head -30; tail -2 gpurun_out/xk1_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_gru.py --H 1024 --T 128 --variants step:0,xc:0,xc:0 --bwd-variants "" --iters 2 > gpurun_out/xk1_bench.log 2>&1
rc=$?; grep variant gpurun_out/xk1_bench.log; [ $rc -ne 0 ] && exit $rc
bash tools/run_xc6.sh
