#!/bin/bash
# GEMM A/B on the step's shapes: persistent vs per-tile kernel vs per-tile without epilogue
# (diagnostic build), plus hipBLASLt on the same shapes. Usage: tools/gemm_diag.sh OUT SHAPES
set -o pipefail
OUT=${1:-gpurun_out/gemm_diag.log}; SHAPES=${2:-input_proj_l1,input_proj_l0,dgrad_l1,square8k}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
{
  echo "== default"; timeout -k 10 120 python $ROOT/tools/bench_gemm.py --shapes $SHAPES --iters 10 || exit 1
  echo "== persist=0"; TT_GEMM_PERSIST=0 timeout -k 10 120 python $ROOT/tools/bench_gemm.py --shapes $SHAPES --iters 10 || exit 1
  echo "== persist=0, no epilogue (diag)"; TT_HIP_LIB=$ROOT/two_towers_amd/lib/libtt_hip_diag.so TT_GEMM_PERSIST=0 \
    timeout -k 10 120 python $ROOT/tools/bench_gemm.py --shapes $SHAPES --iters 10 --regstage 9 || exit 1
  echo "== hipBLASLt"; timeout -k 10 120 python $ROOT/tools/bench_torch_gemm.py || exit 1
} > $OUT 2>&1
