set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 500 python tools/bench_gemm.py --shapes dgrad_l1,c4_proj_l1,c4_dgrad_l1,square8k --iters 3 --rounds 2 \
  --variants="-;gemm_persist_maxk=128" > $OUT/maxk_l.log 2>&1 || exit 3
echo done
