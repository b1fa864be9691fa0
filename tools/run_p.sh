set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gru_persistent.py -q -p no:cacheprovider -rf -x --timeout 120 --timeout-method thread -k paired > $OUT/pytest_pair_t.log 2>&1 || { echo "pair tests failed"; exit 3; }
timeout -k 10 300 python tools/bench_gru.py --bwd-variants "" --iters 3 --variants seq:0,s16:0,seq:0,s16:0 > $OUT/gru_s16_t.log 2>&1 || exit 3
echo done
