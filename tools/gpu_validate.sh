#!/bin/bash
# Full validation on one GPU box: every -m gpu test, smoke, a 2-rank gloo rehearsal of
# bench.py started without a launcher (the N>1 path incl. the overlapped gradient all-reduce), the bench line and a
# rocprofv3 kernel-stats pass. Usage: tools/gpu_validate.sh TAG
set -o pipefail
TAG=${1:-v}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread \
  > $OUT/pytest_$TAG.log 2>&1
rc=$?; echo "pytest exit=$rc" >> $OUT/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest abnormal exit $rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo smoke failed; exit 3; }
TT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --batch 2048 \
  > $OUT/bench_gloo2_$TAG.json 2> $OUT/bench_gloo2_$TAG.err || { echo gloo rehearsal failed; exit 4; }
timeout -k 10 600 python bench.py --timing > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; exit 5; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- python $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_bench_$TAG.json 2> $OUT/prof_bench_$TAG.err || { echo rocprof failed; exit 6; }
echo validate done
