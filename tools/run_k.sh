set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python tools/bench_gemm.py --shapes proj_k128,proj_k320,proj_k1024 --iters 5 --rounds 2 \
  --variants="-;gemm_skew=1;gemm_skew=2;gemm_skew=3;gemm_skew=5" > $OUT/skew_k.log 2>&1 || exit 3
echo done
