"""Summarise a rocprofv3 kernel trace: per-kernel totals and idle gaps between kernels."""
import csv
import glob
import sys
from collections import defaultdict


def main(d, skip_frac=0.4):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = len(rows)
    rows = rows[int(n * skip_frac):]  # drop warm-up
    t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
    busy = defaultdict(float)
    gaps = []
    end = t0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > end:
            gaps.append((s - end, r["Kernel_Name"][:60]))
        end = max(end, e)
        busy[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]] += (e - s)
    span = t1 - t0
    print(f"span {span/1e6:.2f} ms, kernels {len(rows)}, busy(sum) {sum(busy.values())/1e6:.2f} ms, "
          f"idle {sum(g for g, _ in gaps)/1e6:.2f} ms in {len(gaps)} gaps")
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1])[:25]:
        print(f"  {v/1e6:9.3f} ms  {k}")
    gaps.sort(reverse=True)
    print("largest gaps (us) before kernel:")
    for g, k in gaps[:15]:
        print(f"  {g/1e3:8.1f}  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
