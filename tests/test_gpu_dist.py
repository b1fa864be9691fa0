"""Data-parallel path with the HIP kernels: two ranks share the box's GPU over gloo (RCCL
cannot put two ranks on one device; the collectives are the same calls bench.py makes
over RCCL on the 8-GPU node). Each rank holds half of a global batch; the losses all-gather
the doc vectors (global negative pool, labels offset by rank * B), reduce-scatter their
gradient and split the global mean. The per-rank gradients must equal the rows of the
single-process gradients of the whole batch, and the loss must be the same number.

Tolerances (fp32 vectors): loss 1e-5 relative, gradients 1e-4 relative (max-abs over
max); hard-negative indices identical.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, H = 64, 32  # rows per rank, vector width


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make(kind):
    import two_towers_amd as tta
    if kind == "infonce":
        return tta.InfoNCELoss(temperature=0.07)
    return tta.HardNegativeMarginLoss(k=5, margin=0.2)


def _inputs():
    g = torch.Generator().manual_seed(7)
    q = torch.randn(2 * B, H, generator=g)
    d = torch.randn(2 * B, H, generator=g)
    return q, d


def _rank(rank, world, port, kind, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q, d = _inputs()
        ql = q[rank * B:(rank + 1) * B].cuda().requires_grad_(True)
        dl = d[rank * B:(rank + 1) * B].cuda().requires_grad_(True)
        crit = _make(kind)
        loss = crit(ql, dl)
        loss.backward()
        idx = getattr(crit, "last_indices", None)
        out.put((rank, float(loss.detach()), ql.grad.cpu().numpy().copy(), dl.grad.cpu().numpy().copy(),
                 None if idx is None else idx.cpu().numpy().copy()))
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("kind", ["infonce", "hardneg_margin"])
def test_two_ranks_match_single_process(kind):
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, kind, out)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = out.get(timeout=90)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    q, d = _inputs()
    q1 = q.cuda().requires_grad_(True)
    d1 = d.cuda().requires_grad_(True)
    crit = _make(kind)
    loss = crit(q1, d1)
    loss.backward()
    ref_loss = float(loss.detach())
    gq, gd = q1.grad.cpu(), d1.grad.cpu()

    def rel(a, b):
        a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
        return float((a - b).abs().max() / (b.abs().max() + 1e-12))

    for r in range(2):
        l, dq, dd, idx = res[r]
        assert abs(l - ref_loss) <= 1e-5 * abs(ref_loss), (r, l, ref_loss)
        assert rel(dq, gq[r * B:(r + 1) * B]) < 1e-4
        assert rel(dd, gd[r * B:(r + 1) * B]) < 1e-4
        if idx is not None:
            ref_idx = crit.last_indices.cpu().numpy()[r * B:(r + 1) * B]
            assert (idx == ref_idx).all()
