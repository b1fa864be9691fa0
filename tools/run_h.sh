set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider -rf -x --timeout 120 --timeout-method thread -k gemm > $OUT/pytest_gemm_h.log 2>&1 || { echo "gemm tests failed"; exit 3; }
timeout -k 10 600 python tools/bench_gemm.py --shapes input_proj_l0,input_proj_l1,dgrad_l1 --iters 5 --rounds 2 \
  --variants="-;gemm_a3=0;gemm_stream_out=0" > $OUT/gemm_var_h.log 2>&1 || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 300 --timeout-method thread > $OUT/pytest_r03h.log 2>&1; rc=$?; echo "pytest exit=$rc" >> $OUT/pytest_r03h.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest abnormal $rc"; exit $rc; fi
timeout -k 10 300 python bench.py --timing > $OUT/bench_r03h.json 2> $OUT/bench_r03h.err || exit 3
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  TT_HN_MAP=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_hn$m -o p -- python $ROOT/tools/bench_score.py --ops hardneg --hn-shapes 8192x8192x256,8192x65536x256 --iters 20 > $OUT/hn$m.log 2>&1 || exit 3
done
echo done
