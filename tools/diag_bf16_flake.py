"""Repeat test_forward_backward_bf16's body under GRU kernel options and report the worst
gradient cos / relative error against the fp32 oracle (diagnostic for a gradient overflow)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import two_towers_amd as tta  # noqa: E402
from oracle import cpu_ref  # noqa: E402
from two_towers_amd._lib import option  # noqa: E402

DEV = torch.device("cuda")
from two_towers_amd import towers  # noqa: E402

_orig_bwd = towers._gru_layer_bwd
_orig_fwd = towers._gru_layer_fwd if hasattr(towers, "_gru_layer_fwd") else None
LOG = []


def _bwd_probe(cfg, layer, B, T, S, Y, dY, dfinal, packs):
    # inputs of the layer's BPTT and its outputs: report rows holding |x| > 1e6
    torch.cuda.synchronize()
    ins = {}
    for ti in range(len(S)):
        for d in range(2):
            ins["S%d%d" % (ti, d)] = S[ti][d]
        ins["Y%d" % ti] = Y[ti]
        if dY is not None:
            ins["dY%d" % ti] = dY[ti]
    dG, dbih, dbhh = _orig_bwd(cfg, layer, B, T, S, Y, dY, dfinal, packs)
    torch.cuda.synchronize()
    for ti in range(len(dG)):
        ins["dG%d" % ti] = dG[ti]
    for k, x in ins.items():
        bad = (~torch.isfinite(x.float())) | (x.float().abs() > 1e6)
        if bool(bad.any()):
            rows, cols = torch.nonzero(bad, as_tuple=True)
            r = rows.cpu()
            LOG.append({"layer": layer, "buf": k, "n": int(bad.sum()), "rows_bt": sorted(set((int(v) // T, int(v) % T) for v in r[:4000]))[:12],
                        "cols": [int(cols.min()), int(cols.max())]})
    return dG, dbih, dbhh


towers._gru_layer_bwd = _bwd_probe


def run(opts):
    E, h, B, T = 64, int(os.environ.get("HID", "32")), 96, 10
    torch.manual_seed(1)
    m = tta.EnhancedTwoTowerModel(E, h)
    with torch.no_grad():
        for prm in m.parameters():
            prm.copy_(prm.to(torch.bfloat16).float())
    p = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV).eval().set_compute_dtype(torch.bfloat16)
    g = torch.Generator().manual_seed(6)
    q = torch.randn(B, T, E, generator=g).to(torch.bfloat16).float()
    d = torch.randn(B, T, E, generator=g).to(torch.bfloat16).float()
    ctx = [option(k, v) for k, v in opts.items()]
    for c in ctx:
        c.__enter__()
    try:
        qv, dv = m(q.to(DEV), d.to(DEV))
        loss = tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        for c in reversed(ctx):
            c.__exit__(None, None, None)
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    rq, rd = cpu_ref.forward(q, d, pr)
    rl = cpu_ref.infonce(rq, rd)
    rl.backward()
    named = dict(m.named_parameters())
    bad = {}
    for k in pr:
        a, b = named[k].grad.double().cpu(), pr[k].grad.double()
        cos = float((a * b).sum() / (a.norm() * b.norm()))
        frob = float((a - b).norm() / b.norm())
        if not (cos >= 0.998 and frob <= 0.06):
            bad[k] = (round(cos, 4), frob)
    return {"opts": opts, "loss": float(loss), "ref": float(rl), "bad": bad}


nbad = 0
reps = int(os.environ.get("REPS", "30"))
for rep in range(reps):
    for opts in ({}, {"gru_step": 1}):
        r = run(opts)
        if r["bad"] or LOG:
            nbad += 1
            print(json.dumps(r), json.dumps(LOG), flush=True)
        LOG.clear()
print(json.dumps({"lib": os.environ.get("TT_HIP_LIB", "default"), "runs": 2 * reps, "bad_runs": nbad}), flush=True)
