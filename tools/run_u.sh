set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf -x --timeout 200 --timeout-method thread -k "h512 or 1024 or step or reference_size or persistent or bench" > $OUT/pytest_u.log 2>&1 || { echo "tests failed"; exit 3; }
for i in 1 2; do
timeout -k 10 300 python tools/bench_gru.py --H 1024 --T 128 --iters 2 --variants step:0 --bwd-variants "" > $OUT/c4fwd_pf_u$i.log 2>&1 || exit 3
TT_HIP_LIB=$ROOT/two_towers_amd/lib/libtt_hip_exp.so timeout -k 10 300 python tools/bench_gru.py --H 1024 --T 128 --iters 2 --variants step:0 --bwd-variants "" > $OUT/c4fwd_nopf_u$i.log 2>&1 || exit 3
done
echo done
