"""Practical HBM bandwidth on this GPU for the access mixes the step's kernels see
(HIP-event timed torch kernels over 4 GiB buffers): read-only, write-only, copy (1:1),
and a 2:1 read:write stream. Reference points for the roofline fractions in DESIGN.md."""
import json

import torch


def timed(f, iters=10):
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


n = 1 << 30  # 1 Gi fp32 = 4 GiB
a = torch.empty(n, device="cuda")
b = torch.empty(n, device="cuda")
c = torch.empty(n // 2, device="cuda")
a.normal_()
o1 = torch.empty(1024, device="cuda")
res = {}
res["read"] = 4 * n / timed(lambda: torch.sum(a.view(1024, -1), dim=1, out=o1))
res["write"] = 4 * n / timed(lambda: b.fill_(1.0))
res["copy_1to1"] = 8 * n / timed(lambda: b.copy_(a))
res["read2_write1"] = (4 * n + 2 * n) / timed(lambda: torch.add(a[: n // 2], a[n // 2:], out=c))
print(json.dumps({k: round(v / 1e9, 1) for k, v in res.items()} | {"unit": "GB/s"}))
