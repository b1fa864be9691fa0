"""Micro-benchmark of tt_gru_fwd / tt_gru_bwd at the bench shape (4 recurrences:
2 towers x 2 directions), HIP-event timed. Variants via tt_set_option (and TT_GRU_DBG in a -DTT_DIAG build)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from two_towers_amd import _lib  # noqa: E402
from two_towers_amd._lib import GruBwdRec, GruFwdRec, call, set_option, stream_ptr  # noqa: E402


DT = torch.bfloat16


def setup(B, T, H, dev):
    dt = DT
    n = 2
    G = [torch.randn(B * T, 6 * H, device=dev).to(dt) for _ in range(n)]
    whh = [[(torch.randn(3 * H, H, device=dev) * H ** -0.5).to(dt) for _ in range(2)] for _ in range(n)]
    bhn = [[torch.randn(H, device=dev) * 0.1 for _ in range(2)] for _ in range(n)]
    Y = [torch.empty(B * T, 2 * H, device=dev, dtype=dt) for _ in range(n)]
    X1 = [torch.empty(B * T, 2 * H, device=dev, dtype=dt) for _ in range(n)]
    S = [[torch.empty(B * T, 4 * H, device=dev, dtype=dt) for _ in range(2)] for _ in range(n)]
    hs = [torch.empty(2, B, H, device=dev) for _ in range(2 * n)]
    recs = (GruFwdRec * (2 * n))()
    for ti in range(n):
        for d in range(2):
            r = recs[ti * 2 + d]
            r.g = G[ti][:, d * 3 * H:].data_ptr()
            r.whh = whh[ti][d].data_ptr()
            r.bhn = bhn[ti][d].data_ptr()
            r.y = Y[ti][:, d * H:].data_ptr()
            r.x1 = X1[ti][:, d * H:].data_ptr()
            r.save = S[ti][d].data_ptr()
            r.hstate = hs[ti * 2 + d].data_ptr()
            r.dir = d
            r.drop_seed = 7 + ti
            r.drop_col0 = d * H
    keep = (G, whh, bhn, Y, X1, S, hs)
    return recs, keep


def setup_bwd(B, T, H, keep, dev):
    dt = DT
    G, whh, bhn, Y, X1, S, hs = keep
    n = 2
    dY = [torch.randn(B * T, 2 * H, device=dev).to(dt) * 0.01 for _ in range(n)]
    dfin = [torch.randn(B, 2 * H, device=dev) * 0.01 for _ in range(n)]
    dG = [torch.empty(B * T, 8 * H, device=dev, dtype=dt) for _ in range(n)]
    dhs = [torch.empty(2, B, H, device=dev, dtype=dt) for _ in range(2 * n)]
    nbr = _lib.load().tt_gru_bias_rows(B)
    part = [torch.empty(nbr, 4 * H, device=dev) for _ in range(2 * n)]
    recs = (GruBwdRec * (2 * n))()
    for ti in range(n):
        for d in range(2):
            r = recs[ti * 2 + d]
            r.save = S[ti][d].data_ptr()
            r.y = Y[ti][:, d * H:].data_ptr()
            r.dy = dY[ti][:, d * H:].data_ptr()
            r.dfinal = dfin[ti][:, d * H:].data_ptr()
            r.whh = whh[ti][d].data_ptr()
            r.dgx = dG[ti][:, d * 3 * H:].data_ptr()
            r.dgh = dG[ti][:, 6 * H + d * H:].data_ptr()
            r.dhstate = dhs[ti * 2 + d].data_ptr()
            r.dbias_part = part[ti * 2 + d].data_ptr()
            r.dir = d
    return recs, (dY, dfin, dG, dhs, part)


def fwd_call(recs, a, st, ws):
    call("tt_gru_fwd", 0 if DT == torch.float32 else 1, recs, 4, a.B, a.T, a.H, 6 * a.H, 2 * a.H, 0.1,
         ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0, st)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8192)
    ap.add_argument("--T", type=int, default=64)
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--variants", default="xc:0,seq:0",
                    help="kind:dbg[:depth[:skew]]; kind xc (column-split, forced), xcs (write-through exchange), "
                         "xcx (members dealt over XCDs), seq (row-owning), step (per-step)")
    ap.add_argument("--bwd-variants", default="P:0:2", help="rows:dbg:streams[:skew]; rows P (row-owning), S (128x128 "
                    "per-step, `streams` chains), 128 / 64 (per-step 256x256 / 128-row tiles); skew: option gru_bwd_skew")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    a = ap.parse_args()
    global DT
    DT = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    dev = torch.device("cuda")
    recs, keep = setup(a.B, a.T, a.H, dev)
    st = stream_ptr(dev)
    set_option("gru_fwd_xc", 2)
    nb = _lib.load().tt_gru_fwd_ws_size(0 if DT == torch.float32 else 1, 4, a.B, a.T, a.H, 6 * a.H, 2 * a.H)
    ws = torch.zeros(max(nb, 256), dtype=torch.uint8, device=dev) if nb else None
    fwd_call(recs, a, st, ws)  # real S / Y for the backward
    for v in a.bwd_variants.split(","):
        if not v:
            continue
        p = v.split(":")
        rows, dbg, strm, skew = p[0], (p + ["0"])[1], (p + ["0", "2"])[2], (p + ["0", "2", "0"])[3]
        set_option("gru_bwd_skew", int(skew))
        set_option("gru_bwd_persist", 1 if rows == "P" else 0)
        set_option("gru_bwd_big", 0 if rows == "S" else 1)
        set_option("gru_bwd_rows", 128 if rows in ("P", "S") else int(rows))
        os.environ["TT_GRU_DBG"] = dbg  # read only by a -DTT_DIAG build
        set_option("gru_bwd_streams", int(strm))
        brecs, bkeep = setup_bwd(a.B, a.T, a.H, keep, dev)
        f = lambda: call("tt_gru_bwd", 0 if DT == torch.float32 else 1, brecs, 4, a.B, a.T, a.H, 2 * a.H, 8 * a.H, 2 * a.H, st)
        f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            f()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.iters
        print(json.dumps({"bwd_rows": v, "ms": round(ms, 3)}), flush=True)
        del brecs, bkeep
    for v in a.variants.split(","):
        if not v:
            continue
        kind, dbg, *rest = v.split(":")
        depth = rest[:1]
        set_option("gru_fwd_skew", int(rest[1]) if len(rest) > 1 else 0)
        set_option("gru_step", 1 if kind == "step" else 0)
        os.environ["TT_GRU_DBG"] = dbg  # read only by a -DTT_DIAG build
        set_option("gru_depth", int(depth[0]) if depth else 4)
        set_option("gru_fwd_xc", {"xc": 2, "xcs": 6, "xcx": 18}.get(kind, 0))
        f = lambda: fwd_call(recs, a, st, ws if kind.startswith("xc") else None)
        f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            f()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.iters
        gb = a.B * a.T * a.H * 4 * 18 / 1e9
        status = int(ws[:4].view(torch.int32).item()) if ws is not None else 0
        print(json.dumps({"variant": v, "ms": round(ms, 3), "alg_GBs_18B": round(gb / (ms * 1e-3), 1),
                          "xc_status": status}), flush=True)


if __name__ == "__main__":
    main()
