#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Usage: tools/gpu_round.sh TAG [bench args...]   (TT_SKIP_TESTS=1 skips pytest)
set -o pipefail
TAG=${1:-r}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
if [ -z "$TT_SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread \
    > $OUT/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest exit=$rc" >> $OUT/pytest_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest abnormal exit $rc"; exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo smoke failed; exit 3; }
fi
timeout -k 10 900 python bench.py --timing "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; exit 4; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- python $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/prof_bench_$TAG.json 2> $OUT/prof_bench_$TAG.err || { echo rocprof failed; exit 5; }
echo done
