set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
D=$ROOT/two_towers_amd/lib/libtt_hip_diag.so
TT_HIP_LIB=$D timeout -k 10 200 python tools/bench_gemm.py --shapes proj_k128,proj_k320 --iters 5 --regstage 11 --variants="-;gemm_stream_out=0" > $OUT/storeonly_m.log 2>&1 || exit 3
timeout -k 10 100 python tools/bench_hbm.py > $OUT/hbm_m.log 2>&1 || exit 3
echo done
