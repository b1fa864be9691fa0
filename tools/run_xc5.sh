set -o pipefail
mkdir -p gpurun_out
for L in libtt_hip.so libtt_hip_exp1.so libtt_hip_exp6.so libtt_hip.so; do
  TT_HIP_LIB=two_towers_amd/lib/$L timeout -k 10 120 python -u tools/bench_gru.py --variants xc:0,xc:0 --bwd-variants "" --iters 5 > gpurun_out/xc5_$L.log 2>&1 || exit 1
  echo "$L $(grep variant gpurun_out/xc5_$L.log | tr '\n' ' ')"
done
