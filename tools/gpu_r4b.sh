mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hardneg.py tests/test_gpu_dist.py > gpurun_out/r4b_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r4b_pytest.txt
[ $rc -eq 0 ] || exit $rc
bash tools/ab_scan.sh r4b libtt_hip.so > gpurun_out/r4b_scan.txt 2>&1 || exit 1
timeout -k 10 300 python tools/bench_gru.py --variants "xc:0:4:0,xc:0:4:6,xc:0:4:12,xc:0:4:0,xc:0:4:3" --bwd-variants P:0:2:0,P:0:2:10,P:0:2:14,P:0:2:18,P:0:2:24,P:0:2:30,P:0:2:0,P:0:2:14 --iters 5 > gpurun_out/r4b_skew.txt 2>&1 || exit 1
TT_DIST_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4b_bench_rccl1.json 2> gpurun_out/r4b_bench_rccl1.err || exit 1
for d in gpurun_out/abscan_r4b/libtt_hip_1 gpurun_out/abscan_r4b/libtt_hip_2; do python3 tools/kstats.py $(ls $d/*kernel_trace.csv) hn_scan; done
cat gpurun_out/r4b_skew.txt
python3 -c "import json;d=json.load(open('gpurun_out/r4b_bench_rccl1.json'));print(d['value'],d['config'])"
