set -o pipefail
mkdir -p gpurun_out
TT_HIP_LIB=two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 300 python -u tools/diag_xc.py bwd 0 1 2 4 8 16 24 > gpurun_out/xb2_diag.log 2>&1
rc=$?; cat gpurun_out/xb2_diag.log | grep dbg; exit $rc
