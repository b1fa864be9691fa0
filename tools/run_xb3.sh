set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gru_persistent.py -k "backward" > gpurun_out/xb3_pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL" gpurun_out/xb3_pytest.log | head -10; tail -2 gpurun_out/xb3_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_gru.py --variants "" --bwd-variants P:0,X:0,W:0,X:0,P:0 --iters 5 > gpurun_out/xb3_bench.log 2>&1
rc=$?; grep bwd gpurun_out/xb3_bench.log; exit $rc
