# configs[2] A/B of GEMM launch switches on the final build (one box): persistent short-K kernel off,
# 3-slot A ring off, backward skew 0 / 28 (default 14)
mkdir -p gpurun_out
for rep in 1 2; do for v in "base:" "nopersist:TT_GEMM_PERSIST=0" "noa3:TT_GEMM_A3=0" "skew0:TT_GRU_BWD_SKEW=0" "skew28:TT_GRU_BWD_SKEW=28"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4ac_$name.$rep.json 2>> gpurun_out/r4ac_bench.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r4ac_$name.$rep.json')); k=d['kernel_ms_per_step']; print('$name', d['value'], d['ms_per_step'], {n:k[n]['ms_per_step'] for n in ('gru_bwd','input_proj_l1','wgrad_ih','wgrad_hh','dgrad_l1')})
"
done; done
