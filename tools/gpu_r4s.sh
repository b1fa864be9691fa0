# configs[4] (H 1024, T 128, B 8192, bf16) per-step forward: 128- vs 256-row tiles, product ring 2 / 3
mkdir -p gpurun_out
for rep in 1 2; do for v in 256:2 128:2 128:3; do rows=${v%:*}; ring=${v#*:}
  echo "== rows $rows ring $ring"; TT_GRU_FWD_STEP_ROWS=$rows TT_GRU_STEP_RING=$ring timeout -k 10 300 python tools/bench_gru.py --B 8192 --H 1024 --T 128 --iters 2 --variants "step:0" --bwd-variants "" || exit 1
done; done > gpurun_out/r4s_c4fwd.txt 2>&1
grep -v amdgpu gpurun_out/r4s_c4fwd.txt
