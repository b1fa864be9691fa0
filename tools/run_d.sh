set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gru_persistent.py -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread -x > gpurun_out/pytest_r03d.log 2>&1; rc=$?; echo "pytest exit=$rc" >> gpurun_out/pytest_r03d.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest abnormal $rc"; exit $rc; fi
timeout -k 10 300 python tools/bench_gru.py --bwd-variants "" --iters 3 --variants seq:0,wr:0,seq:0,wr:0 > gpurun_out/gru_wr_d.log 2>&1
timeout -k 10 300 python tools/bench_gru.py --bwd-variants "" --iters 3 --H 256 --variants seq:0,wr:0,seq:0,wr:0 >> gpurun_out/gru_wr_d.log 2>&1
timeout -k 10 300 python tools/bench_gemm.py --shapes input_proj_l0,input_proj_l1,dgrad_l1 --iters 5 --rounds 2 \
  --variants="-;gemm_persist=0;gemm_persist=0,gemm_regstage=2;gemm_stream_out=0;gemm_a3=0" > gpurun_out/gemm_var_c.log 2>&1
echo done
