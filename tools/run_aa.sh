set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_hardneg.py -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $OUT/pytest_hn512.log 2>&1 || exit 3
timeout -k 10 300 python tools/bench_score.py --ops hardneg --hn-shapes 8192x8192x256,8192x8192x512,8192x65536x256 > $OUT/score_hn512.log 2>&1 || exit 3
timeout -k 10 300 python tools/bench_score.py --ops hardneg --hn-shapes 8192x8192x256 >> $OUT/score_hn512.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_hn512 -o p -- python $ROOT/tools/bench_score.py --ops hardneg --hn-shapes 8192x8192x512,8192x8192x256,8192x65536x256 > /dev/null 2>&1 || exit 3
echo done
