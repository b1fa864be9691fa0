set -o pipefail
mkdir -p gpurun_out
TT_HIP_LIB=two_towers_amd/lib/libtt_hip_diag.so timeout -k 10 300 python -u tools/diag_xc.py 0 8 2 10 15 > gpurun_out/xc4_diag.log 2>&1
rc=$?; cat gpurun_out/xc4_diag.log | grep dbg; exit $rc
