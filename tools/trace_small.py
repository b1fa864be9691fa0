"""Attribute the configs[2] step's small (non-tt) GPU kernels to their Python call sites:
torch.profiler over 2 steps after warm-up, grouped by the top 6 stack frames."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import two_towers_amd as tta  # noqa: E402
from two_towers_amd import dist as tdp  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, T, h, E, V = 8192, 64, 256, 300, 3_000_000
    torch.manual_seed(1234)
    model = tta.EnhancedTwoTowerModel(E, h).to(dev).set_compute_dtype(torch.bfloat16).train()
    table = (torch.randn(V, E, device=dev) * 0.1).to(torch.bfloat16)
    model.set_embedding_table(table)
    del table
    q = torch.randint(0, V, (B, T), device=dev, dtype=torch.int32)
    d = torch.randint(0, V, (B, T), device=dev, dtype=torch.int32)
    crit = tta.HardNegativeMarginLoss(k=5, margin=0.2, compute_dtype=torch.bfloat16)
    opt = tta.Adam(model.parameters(), lr=1e-3)
    params = list(model.parameters())

    def step():
        opt.zero_grad(set_to_none=True)
        qv, dv = model(q, d)
        loss = crit(qv, dv)
        loss.backward()
        tdp.allreduce_grads(params, None)
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=False) as prof:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_stack_n=6)
    rows = []
    for e in ka:
        dt = getattr(e, "device_time_total", None)
        if dt is None:
            dt = getattr(e, "cuda_time_total", 0)
        if dt <= 0 or e.key.startswith("tt_") or "ProfilerStep" in e.key:
            continue
        rows.append((dt, e.key, e.count, [s for s in e.stack if "two_towers_amd" in s or "trace_small" in s][:4]))
    rows.sort(key=lambda r: -r[0])
    for dt, key, cnt, st in rows[:40]:
        print(f"{dt / 2 / 1e3:8.3f} ms/step  x{cnt / 2:5.1f}  {key[:60]}")
        for s in st:
            print("            ", s)


if __name__ == "__main__":
    main()
