"""Per-kernel duration summary of a rocprofv3 kernel trace: python tools/kstats.py trace.csv [substr...]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pats = sys.argv[2:]
agg = collections.OrderedDict()
for r in rows:
    n = r["Kernel_Name"]
    if pats and not any(p in n for p in pats):
        continue
    key = (re.sub(r"^void |\(anonymous namespace\)::", "", n).split("(")[0][-60:], r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size"))
    agg.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for (n, g), v in agg.items():
    v.sort()
    print(f"{n:62s} grid {g:>8s} n {len(v):3d} med {v[len(v)//2]:9.2f} us  min {v[0]:9.2f}")
