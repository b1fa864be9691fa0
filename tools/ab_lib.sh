#!/bin/bash
# A/B of the experiment library (lib/libtt_hip_exp.so) against the product library over one tool
# command, alternating twice in one call. Usage: tools/ab_lib.sh OUT -- command args...
set -o pipefail
OUT=$1; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
{ for rep in 1 2; do for lib in libtt_hip.so libtt_hip_exp.so; do
  echo "== $lib"; TT_HIP_LIB=$ROOT/two_towers_amd/lib/$lib timeout -k 10 200 "$@" || exit 1
done; done; } > $OUT 2>&1
