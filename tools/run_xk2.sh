set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gru_persistent.py -k "h1024" > gpurun_out/xk2_pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL" gpurun_out/xk2_pytest.log | head -10; tail -2 gpurun_out/xk2_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_gru.py --H 1024 --T 128 --variants step:0,xc:0,xc:0 --bwd-variants "" --iters 2 > gpurun_out/xk2_bench.log 2>&1
rc=$?; grep variant gpurun_out/xk2_bench.log; exit $rc
