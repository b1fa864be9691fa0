mkdir -p gpurun_out
timeout -k 10 900 python bench.py --cpu-only --cpu-batch 8192 --cpu-steps 2 --cpu-warmup 1 > gpurun_out/r4_cpu_b8192.json 2> gpurun_out/r4_cpu_b8192.err || exit 1
cat gpurun_out/r4_cpu_b8192.json
