#!/bin/bash
# Per-kernel register / LDS use of one HIP source (device compile only):
# tools/kres.sh two_towers_amd/csrc/tt_gru.hip [name-substring]
src=$1; pat=${2:-.}
cd "$(dirname "$src")" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC --offload-device-only \
  -c "$(basename "$src")" -o /tmp/kres_dev.o -Rpass-analysis=kernel-resource-usage $EXTRA 2>&1 | python3 -c '
import re, sys
cur = None
rows = {}
for ln in sys.stdin:
    m = re.search(r"remark: (.*?): (\S+) \[", ln)
    if not m: continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name": cur = v; rows[cur] = {}
    elif cur: rows[cur][k] = v
for n, r in rows.items():
    if re.search(sys.argv[1], n):
        g = lambda k: r.get(k)
        print("%-70s vgpr %s agpr %s spill %s lds %s occ %s" % (n[:70], g("VGPRs"), g("AGPRs"), g("VGPRs Spill"), g("LDS Size [bytes/block]"), g("Occupancy [waves/SIMD]")))
' "$pat"
