"""Per-kernel mean of every collected counter across rocprofv3 --pmc passes
(usage: pmc_summary.py DIR [STEPS_TOTAL] -> JSON on stdout).
FETCH_SIZE / WRITE_SIZE are KB; on gfx950 FETCH_SIZE counts half the bytes of wide
coalesced reads (MI355X_MICROARCH.md §HBM), so hbm_bytes = 2*FETCH + WRITE (x1024)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:110]


def main(d, steps_total=None):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes_est"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
        if steps_total:
            m["dispatches_per_step"] = m["dispatches"] / float(steps_total)
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            m["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        out[k] = m
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
