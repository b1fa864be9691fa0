set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gru_persistent.py -k "column_split" > gpurun_out/xb1_pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|tower 0 block 0|bias" gpurun_out/xb1_pytest.log | head -40; tail -3 gpurun_out/xb1_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_gru.py --variants "" --bwd-variants P:0,X:0,X:0 --iters 5 > gpurun_out/xb1_bench.log 2>&1
rc=$?; cat gpurun_out/xb1_bench.log | grep bwd; exit $rc
