#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Usage: tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > $OUT/pytest_$TAG.log 2>&1
rc=$?; echo "pytest exit=$rc" >> $OUT/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest abnormal exit $rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo smoke failed; exit 3; }
timeout -k 10 900 python bench.py --timing "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; exit 4; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o prof -- python $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/prof_bench_$TAG.json 2> $OUT/prof_bench_$TAG.err || { echo rocprof failed; exit 5; }
echo done
