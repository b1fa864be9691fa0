mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4d_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r4d_pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4d_smoke.txt 2>&1 || exit 1
timeout -k 10 300 python tools/bench_gru.py --variants "" --bwd-variants P:0:2:0,P:0:2:14,P:0:2:-7,P:0:2:-5,P:0:2:-9,P:0:2:14,P:0:2:-7 --iters 5 > gpurun_out/r4d_skew.txt 2>&1 || exit 1
cat gpurun_out/r4d_skew.txt
for v in "" "TT_GRU_BWD_STREAMS=1" "TT_GRU_FWD_STEP_ROWS=256" "TT_GRU_FWD_STEP_ROWS=128"; do
  env $v timeout -k 10 300 python bench.py --batch 1024 --dtype fp32 --loss infonce --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r4d_bench_c1.json 2>> gpurun_out/r4d_bench.err || exit 1
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/r4d_bench_c1.json')); k=d['kernel_ms_per_step']; print('c1 $v', d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in k})
"
done
# gru_bwd_rows phase diagnostics (diag build: 1 no GEMM, 2 no epilogue loads, 4 no stores), skew 14 default
TT_HIP_LIB=two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 300 python tools/bench_gru.py --variants "" --bwd-variants P:0:2:14,P:1:2:14,P:2:2:14,P:4:2:14,P:6:2:14,P:7:2:14,P:0:2:0,P:1:2:0,P:6:2:0 --iters 5 > gpurun_out/r4d_bwd_diag.txt 2>&1 || exit 1
cat gpurun_out/r4d_bwd_diag.txt
# hn_scan block maps: 0 split per XCD (default), 1 row tile per XCD, 2 row halves x split quarters per XCD
for rep in 1 2; do
timeout -k 10 200 python tools/bench_score.py --ops hardneg --iters 50 --hn-shapes 8192x8192x256,8192x65536x256 --variants "map1=hn_map=1;map2=hn_map=2" >> gpurun_out/r4d_hnmap.txt 2>&1 || exit 1
done
cat gpurun_out/r4d_hnmap.txt
# hn_scan query prologue overlapped with tile 0 (libtt_hip, HN_PIPE_Q=1) vs retired up front (libtt_hip_exp, HN_PIPE_Q=0)
bash tools/ab_scan.sh r4d libtt_hip.so libtt_hip_exp.so > gpurun_out/r4d_scan.txt 2>&1 || exit 1
cat gpurun_out/r4d_scan.txt
