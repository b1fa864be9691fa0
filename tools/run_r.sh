set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python tools/bench_gru.py --bwd-variants "" --iters 3 --variants seq:0,tm:0,seq:0,tm:0 > $OUT/gru_tm_r.log 2>&1 || exit 3
echo done
