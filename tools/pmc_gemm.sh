#!/bin/bash
# Stall-breakdown and cache counters over tools/bench_gemm.py (one counter group per pass).
# Usage: tools/pmc_gemm.sh TAG SHAPES [bench_gemm args...]
set -o pipefail
TAG=${1:-x}; SHAPES=${2:-square8k}; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmcg_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o p -- \
    python $ROOT/tools/bench_gemm.py --shapes $SHAPES --iters 2 "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python $ROOT/tools/pmc_summary.py $OUT > $OUT/summary.json
echo pmc done
