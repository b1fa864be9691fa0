"""Where gru_fwd_wr differs from the per-step forward (diagnostic, GPU)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from test_gpu_gru_persistent import _inputs, _run  # noqa: E402
from two_towers_amd._lib import option  # noqa: E402


def main():
    for (H, B, T) in [(512, 1000, 12), (512, 8192, 8), (512, 8192, 64), (256, 8192, 64), (512, 2048, 64)]:
        G, whh, bhn = _inputs(2, B, T, H, seed=H + B + T)
        s = _run(2, B, T, H, G, whh, bhn, 0.1, step=1)
        with option("gru_fwd_wr", 1):
            p = _run(2, B, T, H, G, whh, bhn, 0.1, step=0)
        # Y of tower 0: [B*T, 2H] -> [B, T, 2, H]
        ys, yp = s[1][0].view(B, T, 2, H), p[1][0].view(B, T, 2, H)
        d = (ys.view(torch.int16) != yp.view(torch.int16))
        out = {"H": H, "B": B, "T": T, "frac": float(d.float().mean())}
        if d.any():
            for dr in range(2):
                dd = d[:, :, dr, :]
                steps = dd.any(dim=2).any(dim=0).nonzero().flatten().tolist()
                # first differing step index (in processing order) per row
                rows = dd.any(dim=2).any(dim=1).nonzero().flatten()
                out[f"dir{dr}_rows"] = int(rows.numel())
                out[f"dir{dr}_rows_mod64"] = sorted(set((rows % 64).tolist()))[:20]
                out[f"dir{dr}_wg"] = sorted(set((rows // 64).tolist()))[:20]
                tt = steps if dr == 0 else [T - 1 - x for x in steps]
                out[f"dir{dr}_first_steps"] = sorted(tt)[:10]
                # units of the first differing step
                s0 = min(tt)
                t0 = s0 if dr == 0 else T - 1 - s0
                u = dd[:, t0, :].any(dim=0).nonzero().flatten().tolist()
                out[f"dir{dr}_units_first"] = u[:40]
                out[f"dir{dr}_rows_first"] = dd[:, t0, :].any(dim=1).nonzero().flatten().tolist()[:20]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
