set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python tools/bench_gemm.py --shapes input_proj_l0,input_proj_l1 --iters 5 --rounds 2 --variants="-;gemm_stream_out=2;gemm_stream_out=3;gemm_stream_out=0" > $OUT/pol_n.log 2>&1 || exit 3
echo done
