#!/bin/bash
# A/B of one tt option over tools/bench_gemm.py shapes, alternating 0/1 twice in one call.
# Usage: tools/ab_gemm_opt.sh ENVVAR SHAPES OUT
set -o pipefail
V=$1; SHAPES=$2; OUT=$3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
{ for rep in 1 2; do for x in 0 1; do
  echo "== $V=$x"; env $V=$x timeout -k 10 150 python $ROOT/tools/bench_gemm.py --shapes $SHAPES --iters 10 || exit 1
done; done; } > $OUT 2>&1
