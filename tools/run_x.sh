set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread -k "interleaved or persistent" > $OUT/pytest_il_x.log 2>&1; echo "rc=$?" >> $OUT/pytest_il_x.log
timeout -k 10 300 python tools/bench_gemm.py --shapes input_proj_l0,input_proj_l1 --no-bias --iters 5 --rounds 2 --variants="-;gemm_il=1" > $OUT/il_x.log 2>&1 || exit 3
echo done
