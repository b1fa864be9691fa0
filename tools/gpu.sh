#!/bin/bash
# Rebuild libtt_hip.so locally, then run a command on the GPU box via gpurun.
# Usage: tools/gpu.sh TIMEOUT 'command'
set -e
cd /root/repo
make -C two_towers_amd/csrc -j8 >/dev/null
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
