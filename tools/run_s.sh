set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_fwd_s
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM" \
           "SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_BUSY_max"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o p -- \
    python $ROOT/tools/bench_gru.py --bwd-variants "" --iters 2 --variants seq:0 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo pmc done
