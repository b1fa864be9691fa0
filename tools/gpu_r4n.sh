# Final-build validation: full GPU suite, smoke, configs[2] bench (x2), rocprofv3 kernel
# stats (column-split forward launched plainly: profiles/r04_rocprof_crash_k.txt), the
# configs[1] and configs[4] lines
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4n_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r4n_pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4n_smoke.txt 2>&1 || exit 1
grep smoke gpurun_out/r4n_smoke.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4n_bench_$i.json 2>> gpurun_out/r4n_bench.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r4n_bench_$i.json')); k=d['kernel_ms_per_step']; print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], {n:k[n]['ms_per_step'] for n in k})
"
done
timeout -k 10 300 python bench.py --batch 1024 --dtype fp32 --loss infonce --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4n_bench_c1.json 2>> gpurun_out/r4n_bench.err || exit 1
timeout -k 10 600 python bench.py --hidden 512 --seq 128 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4n_bench_c4.json 2>> gpurun_out/r4n_bench.err || exit 1
python3 -c "
import json
for f in ('c1','c4'):
    d=json.load(open('gpurun_out/r4n_bench_'+f+'.json')); k=d['kernel_ms_per_step']; print(f, d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
cd /tmp && export TMPDIR=/tmp
TT_GRU_XC_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4n_prof -o p -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r4n_prof.log 2>&1 || exit 1
echo prof ok
