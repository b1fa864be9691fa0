set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_path.py tests/test_gpu_model.py -v -s --timeout 250 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pt_d.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pt_d.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --timing --no-cpu-baseline --hidden 512 --seq 128 --steps 5 --warmup 2 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o prof -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --hidden 512 --seq 128 --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_c4.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_c4.err || exit 5
