set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/pytest_r03z.log 2>&1; rc=$?; echo "pytest exit=$rc" >> $OUT/pytest_r03z.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest abnormal $rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_r03z.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --timing > $OUT/bench_r03z.json 2> $OUT/bench_r03z.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r03z -o prof -- python $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_bench_r03z.json 2> $OUT/prof_bench_r03z.err || exit 3
echo done
