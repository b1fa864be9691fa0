#!/bin/bash
# A/B of one tt option over tools/bench_gru.py (forward seq + row-owning backward): values A and B
# alternating twice. Usage: tools/ab_gru_opt.sh ENVVAR "A B" OUT [bench_gru args...]
set -o pipefail
V=$1; VALS=$2; OUT=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
{ for rep in 1 2; do for x in $VALS; do
  echo "== $V=$x"; env $V=$x timeout -k 10 150 python $ROOT/tools/bench_gru.py --variants seq:0 --bwd-variants P:0:2 "$@" || exit 1
done; done; } > $OUT 2>&1
