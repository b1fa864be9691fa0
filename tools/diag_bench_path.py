"""Per-parameter gradient error of the bf16 bench configuration vs the fp32 oracle
(tests/test_gpu_bench_path.py setup), sorted worst first. Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tests.test_gpu_bench_path as tb  # noqa: E402
import two_towers_amd as tta  # noqa: E402
from oracle import cpu_ref  # noqa: E402

for drop_p in (0.0, 0.1):
    for mseed in (31, 41):
        m, p = tb._model(mseed)
        m.train() if drop_p > 0 else m.eval()
        g = torch.Generator().manual_seed(32)
        q = tb._bf16(torch.randn(tb.B, tb.T, tb.E, generator=g) * 0.5)
        d = tb._bf16(torch.randn(tb.B, tb.T, tb.E, generator=g) * 0.5)
        torch.manual_seed(33)
        qv, dv = m(q.cuda(), d.cuda())
        loss = tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv)
        loss.backward()
        torch.manual_seed(33)
        seeds = [int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) for _ in range(2)] if drop_p > 0 else [0, 0]
        rq, rd = cpu_ref.forward(q, d, p, drop_p=drop_p, seeds=seeds)
        rl = cpu_ref.infonce(rq, rd)
        rl.backward()
        rows = []
        for k, pr in p.items():
            a, b = dict(m.named_parameters())[k].grad.double().cpu(), pr.grad.double()
            rows.append((float((a - b).norm() / b.norm()), float((a * b).sum() / (a.norm() * b.norm())), k))
        rows.sort(reverse=True)
        print(f"drop {drop_p} seed {mseed}: loss {float(loss):.6f} vs {float(rl):.6f}", flush=True)
        for r in rows[:8]:
            print(f"   {r[2]:40s} rel {r[0]:.4f} cos {r[1]:.5f}", flush=True)
