set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_gemm.py --shapes input_proj_l0,input_proj_l1,dgrad_l1 --iters 5 --rounds 2 \
  --variants="-;gemm_persist=0;gemm_persist=0,gemm_regstage=2;gemm_stream_out=0;gemm_a3=0" > gpurun_out/gemm_var_c.log 2>&1
echo done
