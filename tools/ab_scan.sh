#!/bin/bash
# hn_scan A/B: rocprofv3 kernel stats over tools/bench_score.py hardneg for each library.
# Usage: tools/ab_scan.sh TAG [lib.so ...]   (default: libtt_hip.so libtt_hip_exp.so)
set -o pipefail
TAG=${1:-x}; shift
LIBS=${@:-libtt_hip.so libtt_hip_exp.so}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/abscan_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do for lib in $LIBS; do
  TT_HIP_LIB=$ROOT/two_towers_amd/lib/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/${lib%.so}_$rep -o p -- python $ROOT/tools/bench_score.py --ops hardneg --iters 20 \
    --hn-shapes 8192x8192x256,8192x65536x256 > $OUT/${lib%.so}_$rep.log 2>&1 || { echo "prof $lib $rep failed"; exit 1; }
done; done
python - $OUT <<'PY'
import csv, glob, sys
for d in sorted(glob.glob(sys.argv[1] + "/libtt*/")):
    f = glob.glob(d + "**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "hn_" in r["Name"]:
            print(d.rstrip("/").split("/")[-1], r["Name"].split("(")[0][-28:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
