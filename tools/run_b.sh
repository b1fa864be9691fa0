set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread -x > gpurun_out/pytest_r03b.log 2>&1; echo "pytest exit=$?" >> gpurun_out/pytest_r03b.log
TT_HIP_LIB=two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 300 python tools/bench_gru.py --bwd-variants "" --iters 3 --variants seq:0,seq:1,seq:2,seq:4,seq:8,seq:16,seq:24,seq:32,seq:36,seq:28,seq:0 > gpurun_out/gru_diag_b.log 2>&1
TT_HIP_LIB=two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 300 python tools/diag_fwd_stamps.py >> gpurun_out/gru_diag_b.log 2>&1
echo done
