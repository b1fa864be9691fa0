set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_r03f.log 2>&1; rc=$?; echo "pytest exit=$rc" >> gpurun_out/pytest_r03f.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest abnormal $rc"; exit $rc; fi
timeout -k 10 300 python tools/bench_gru.py --bwd-variants "" --iters 3 --variants seq:0,wr:0,seq:0,wr:0 > gpurun_out/gru_wr_f.log 2>&1
timeout -k 10 600 python tools/bench_gemm.py --shapes input_proj_l0,input_proj_l1,dgrad_l1 --iters 5 --rounds 2 \
  --variants="-;gemm_persist=0;gemm_persist=0,gemm_regstage=2;gemm_stream_out=0;gemm_a3=0" > gpurun_out/gemm_var_f.log 2>&1
timeout -k 10 300 python bench.py --timing > gpurun_out/bench_r03f.json 2> gpurun_out/bench_r03f.err
echo done
