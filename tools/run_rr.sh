set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/bench_gru.py --B 8192 --T 64 --H 512 --bwd-variants "" --check seq:rr2 --variants "seq:0,rr:0,rr2:0,rr3:0" > gpurun_out/rr_c.log 2>&1 || exit 3
TT_HIP_LIB=two_towers_amd/lib/libtt_hip_exp.so timeout -k 10 240 python -u tools/bench_gru.py --B 8192 --T 64 --H 512 --bwd-variants "" --variants "seq:0,rr:0,rr2:0,rr3:0" >> gpurun_out/rr_c.log 2>&1 || exit 4
