#!/bin/bash
# PMC passes over a short bench.py run (each counter group in its own pass, per
# MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass). Then summarise
# per-kernel average counters -> gpurun_out/pmc_$TAG/summary.json
set -o pipefail
TAG=${1:-x}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o p -- \
    python $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
# 1 warm-up + 2 timed steps per pass -> dispatches per training step
python $ROOT/tools/pmc_summary.py $OUT 3 > $OUT/summary.json
echo pmc done
