set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread -k "big_tiles" > $OUT/pytest_w4_v.log 2>&1; echo "pytest rc=$?" >> $OUT/pytest_w4_v.log
timeout -k 10 500 python tools/bench_gemm.py --shapes square8k,input_proj_l1,dgrad_l1,wgrad_ih1,wgrad_hh --iters 3 --rounds 2 \
  --variants="gemm_persist=0;gemm_persist=0,gemm_w4=1" > $OUT/w4_v.log 2>&1 || exit 3
echo done
