set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_path.py -v -s --timeout 250 --timeout-method thread -p no:cacheprovider -rf -k "row_owning or bench_config or big_tile or h512" > gpurun_out/pt_f.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pt_f.log
if [ $rc -gt 1 ]; then exit $rc; fi
TT_HIP_LIB=two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 300 python tools/bench_gru.py --bwd-variants "128:0,P:0,P:1,P:2,P:4,P:6,P:7,128:0,P:0" --variants "" --iters 3 > gpurun_out/bg_f.log 2>&1 || exit 3
