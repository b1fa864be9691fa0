set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_wr.py > gpurun_out/diag_wr_e.log 2>&1
echo done
