# product ring: bit-identity incl. 128-row backward tiles at 4 stages; fp32 recurrence at B 2048 (ring on / off)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ring.py > gpurun_out/r4aa_pytest.txt 2>&1; rc=$?; tail -6 gpurun_out/r4aa_pytest.txt
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for ring in 4 2; do echo "== ring $ring B 2048"; TT_GRU_STEP_RING=$ring timeout -k 10 200 python tools/bench_gru.py --dtype fp32 --B 2048 --H 512 --T 64 --iters 3 --variants "step:0" --bwd-variants "128:0:2,64:0:2" || exit 1; done; done > gpurun_out/r4aa_b2048.txt 2>&1
grep -v amdgpu gpurun_out/r4aa_b2048.txt
