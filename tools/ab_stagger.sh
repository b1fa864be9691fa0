# A/B of the staggered W_hh block order in the persistent GRU forward (env TT_GRU_STAGGER).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_model.py -k "persistent" > gpurun_out/ab_test.log 2>&1; echo "test rc=$?"; tail -n 3 gpurun_out/ab_test.log
for s in 0 1 0 1; do TT_GRU_STAGGER=$s timeout -k 10 200 python tools/bench_gru.py --iters 5 --bwd-variants "" > gpurun_out/ab_gru_$s.log 2>&1 || { echo gru $s failed; exit 4; }; echo "stagger $s: $(tail -n 1 gpurun_out/ab_gru_$s.log)"; done
TT_GRU_STAGGER=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_bench1.json 2> gpurun_out/ab_bench1.err || exit 5
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_bench0.json 2> gpurun_out/ab_bench0.err || exit 5
for f in gpurun_out/ab_bench0.json gpurun_out/ab_bench1.json; do python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],d['kernel_ms_per_step']['gru_fwd'])" $f; done
