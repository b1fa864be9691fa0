set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
D=$ROOT/two_towers_amd/lib/libtt_hip_diag.so
for rs in 0 12 9; do
TT_HIP_LIB=$D timeout -k 10 200 python tools/bench_gemm.py --shapes proj_k128,proj_k320,proj_k1024 --iters 5 --regstage $rs > $OUT/loose_w_$rs.log 2>&1 || exit 3
done
echo done
