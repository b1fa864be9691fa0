set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
TT_HIP_LIB=$ROOT/two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 400 python tools/bench_gru.py --bwd-variants "" --iters 2 --variants seq:0,seq:1,seq:2,seq:3,seq:16,seq:19,seq:8,seq:27,seq:31,seq:0 > $OUT/gru_diag_y.log 2>&1 || exit 3
echo done
