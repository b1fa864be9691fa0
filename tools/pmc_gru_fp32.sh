#!/bin/bash
# Counter passes over the fp32 per-step GRU kernels at configs[1] (tools/bench_gru.py --dtype fp32),
# one counter group per pass -> gpurun_out/pmcg_TAG/summary.json
set -o pipefail
TAG=${1:-x}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmcg_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o p -- \
    python $ROOT/tools/bench_gru.py --dtype fp32 --B 1024 --H 512 --T 64 --iters 1 --variants "step:0" --bwd-variants "64:0:2" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python $ROOT/tools/pmc_summary.py $OUT > $OUT/summary.json
echo pmc done
