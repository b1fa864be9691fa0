set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_path.py tests/test_gpu_dist.py tests/test_gpu_golden.py -v --timeout 200 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pt_c.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pt_c.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/diag_bench_path.py > gpurun_out/diag_bp.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --timing --no-cpu-baseline > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || exit 4
tail -2 gpurun_out/pt_c.log
