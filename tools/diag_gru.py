"""Compare tt_gru_fwd persistent vs per-step outputs element-wise (diagnostics)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_gru import setup  # noqa: E402
from two_towers_amd._lib import call, set_option, stream_ptr  # noqa: E402

for (B, T, H) in [(200, 7, 128), (200, 7, 512), (128, 3, 128)]:
    torch.manual_seed(0)
    recs, keep = setup(B, T, H, torch.device("cuda"))
    G, whh, bhn, Y, X1, S, hs = keep
    outs = []
    for step in ("1", "0"):
        set_option("gru_step", int(step))
        for y in Y: y.zero_()
        for s2 in S:
            for s in s2: s.zero_()
        call("tt_gru_fwd", 1, recs, 4, B, T, H, 6 * H, 2 * H, 0.1, stream_ptr(torch.device("cuda")))
        torch.cuda.synchronize()
        outs.append(([y.float().clone() for y in Y], [[s.float().clone() for s in s2] for s2 in S]))
    (y0, s0), (y1, s1) = outs
    for ti in range(2):
        d = (y0[ti] - y1[ti]).abs().reshape(B, T, 2 * H)
        bad = (d > 1e-6).nonzero()
        print(B, T, H, "tower", ti, "Y maxdiff", float(d.max()), "nbad", bad.shape[0])
        if bad.shape[0]:
            print("  rows", sorted(set(bad[:, 0].tolist()))[:20], "t", sorted(set(bad[:, 1].tolist())),
                  "cols", sorted(set(bad[:, 2].tolist()))[:40])
        for dd in range(2):
            ds = (s0[ti][dd] - s1[ti][dd]).abs().reshape(B, T, 4, H)
            bad = (ds > 1e-6).nonzero()
            print("   S dir", dd, "maxdiff", float(ds.max()), "nbad", bad.shape[0],
                  "q", sorted(set(bad[:, 2].tolist())) if bad.shape[0] else "")
