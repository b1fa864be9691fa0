#!/bin/bash
# hn_scan A/B: rocprofv3 kernel traces over tools/bench_score.py hardneg for each library,
# summarised per (library run, kernel, grid) as the median traced dispatch duration (the two
# shapes launch the same kernels, so the stats file alone would average them together).
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
import collections, csv, glob, sys
for d in sorted(glob.glob(sys.argv[1] + "/libtt*/")):
    f = glob.glob(d + "**/*kernel_trace.csv", recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "hn_" in r["Kernel_Name"]:
            name = r["Kernel_Name"].split("::")[-1].split("(")[0]
            agg[(name, r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (name, grid), v in sorted(agg.items()):
        v.sort()
        print(d.rstrip("/").split("/")[-1], name, "grid", grid, len(v), "median us", round(v[len(v) // 2], 2))
PY
