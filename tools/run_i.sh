set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
SH=proj_k128,proj_k192,proj_k320,proj_k512,proj_k768,proj_k1024,proj_k1536
timeout -k 10 300 python tools/bench_gemm.py --shapes $SH --iters 5 --rounds 2 --variants="-" > $OUT/ksweep_i.log 2>&1 || exit 3
timeout -k 10 300 python tools/bench_gemm.py --shapes $SH --iters 5 --lda-pad -1 > $OUT/ksweep_l2a_i.log 2>&1 || exit 3
TT_HIP_LIB=$ROOT/two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 300 python tools/bench_gemm.py --shapes $SH --iters 5 --regstage 9 > $OUT/ksweep_nostore_i.log 2>&1 || exit 3
TT_HIP_LIB=$ROOT/two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 300 python tools/bench_gemm.py --shapes $SH --iters 5 --regstage 9 --lda-pad -1 > $OUT/ksweep_nostore_l2a_i.log 2>&1 || exit 3
echo done
