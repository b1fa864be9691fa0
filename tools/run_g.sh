set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  TT_HN_MAP=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_hn$m -o p -- python $ROOT/tools/bench_score.py --ops hardneg --hn-shapes 8192x8192x256,8192x65536x256 --iters 20 > $OUT/hn$m.log 2>&1 || exit 3
done
echo done
