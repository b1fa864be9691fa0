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


# ------------------------------------------------------------------ full training step
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dp_golden():
    import numpy as np
    return np.load(os.path.join(GOLD, "dp_step.npz"), allow_pickle=False)


def _dp_model(z):
    import two_towers_amd as tta
    m = tta.EnhancedTwoTowerModel(16, 8)
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w.")})
    return m.cuda().eval()


def _step_rank(rank, world, port, kind, overlap, out, backend="gloo"):
    """train_enhanced.py:58-63 on this rank's rows: zero_grad, forward, loss (global
    negative pool), backward, gradient all-reduce, Adam. overlap: the tower gradients are
    summed inside the backward (set_process_group(..., overlap_grad_allreduce=True)) and
    allreduce_grads sums only the rest; otherwise allreduce_grads sums everything.
    backend "nccl" (RCCL) with world 1: TT_DIST_FORCE=1 makes every collective run anyway."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        os.environ["TT_DIST_FORCE"] = "1"
        torch.cuda.set_device(0)
        torch.distributed.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import two_towers_amd as tta
        from two_towers_amd import dist as tdp
        z = _dp_golden()
        n = z["q"].shape[0] // world
        q = torch.from_numpy(z["q"][rank * n:(rank + 1) * n]).cuda()
        d = torch.from_numpy(z["d"][rank * n:(rank + 1) * n]).cuda()
        m = _dp_model(z).set_process_group(None, overlap_grad_allreduce=overlap)
        opt = tta.Adam(m.parameters(), lr=1e-3)
        crit = tta.InfoNCELoss() if kind == "infonce" else tta.HardNegativeMarginLoss(k=5, margin=0.2)
        opt.zero_grad()
        loss = crit(*m(q, d))
        loss.backward()
        tdp.allreduce_grads(list(m.parameters()))
        grads = {k: p.grad.cpu().numpy().copy() for k, p in m.named_parameters()}
        opt.step()
        w1 = {k: v.cpu().numpy().copy() for k, v in m.state_dict().items()}
        idx = getattr(crit, "last_indices", None)
        out.put((rank, float(loss.detach()), grads, w1, None if idx is None else idx.cpu().numpy().copy()))
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,overlap", [(2, False), (2, True), (4, True)])
@pytest.mark.parametrize("kind", ["infonce", "hardneg"])
def test_dp_train_step_matches_reference_global_batch(kind, world, overlap):
    """a data-parallel step over the 256 rows of dp_step.npz
    (256 / world per rank; world 4 with the hard-negative margin loss is the configs[3]
    composition: every rank mines its rows against the all-gathered global pool)
    reproduces the reference's single-process step on all 256: loss 1e-5 relative, every
    all-reduced gradient 2e-3 (max-abs over max, the fp32 tolerance of the golden tests),
    weights after Adam within 1 % of lr, and the mined hard negatives of each rank equal
    the reference's rows. Both gradient reductions: in the backward (overlap) and after."""
    import numpy as np
    z = _dp_golden()
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_step_rank, args=(r, world, port, kind, overlap, out)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = out.get(timeout=180)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = z["q"].shape[0] // world
    for r in range(world):
        loss, grads, w1, idx = res[r]
        ref = float(z[f"{kind}.loss"])
        assert abs(loss - ref) <= 1e-5 * abs(ref), (r, loss, ref)
        for k, g in grads.items():
            gr = z[f"{kind}.g.{k}"]
            assert float(np.abs(g - gr).max()) <= 2e-3 * float(np.abs(gr).max()) + 1e-9, (r, k)
        for k, w in w1.items():
            assert float(np.abs(w - z[f"{kind}.w1.{k}"]).max()) <= 1e-5, (r, k)
        if idx is not None:
            assert (idx == z["hardneg.idx"][r * n:(r + 1) * n]).all()


@pytest.mark.parametrize("kind", ["infonce", "hardneg"])
def test_rccl_one_rank_train_step_matches_reference(kind):
    """The DP step's collectives over RCCL ("nccl") on the box's one GPU: a one-rank process
    group with TT_DIST_FORCE=1, so the doc-vector all-gather, its reduce-scatter, the loss
    all-reduce and the overlapped + bucketed gradient all-reduces all execute as RCCL
    kernels (the 8-GPU node runs the same calls). Must reproduce the reference's
    single-process step on dp_step.npz exactly as the gloo worlds do."""
    import numpy as np
    z = _dp_golden()
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    p = ctx.Process(target=_step_rank, args=(0, 1, _port(), kind, True, out, "nccl"))
    p.start()
    _, loss, grads, w1, idx = out.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    ref = float(z[f"{kind}.loss"])
    assert abs(loss - ref) <= 1e-5 * abs(ref), (loss, ref)
    for k, g in grads.items():
        gr = z[f"{kind}.g.{k}"]
        assert float(np.abs(g - gr).max()) <= 2e-3 * float(np.abs(gr).max()) + 1e-9, k
    for k, w in w1.items():
        assert float(np.abs(w - z[f"{kind}.w1.{k}"]).max()) <= 1e-5, k
    if idx is not None:
        assert (idx == z["hardneg.idx"]).all()


def _drop_rank(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import two_towers_amd as tta
        from two_towers_amd import dist as tdp
        z = _dp_golden()
        n = z["q"].shape[0] // world
        m = _dp_model(z).train()  # GRU dropout 0.1 between the layers
        torch.manual_seed(40)  # same dropout seeds on every rank, as in bench.py / train.py
        qv, dv = m(torch.from_numpy(z["q"][rank * n:(rank + 1) * n]).cuda(),
                   torch.from_numpy(z["d"][rank * n:(rank + 1) * n]).cuda())
        tta.InfoNCELoss()(qv, dv).backward()
        tdp.allreduce_grads(list(m.parameters()))
        out.put((rank, qv.detach().cpu().numpy().copy(),
                 {k: p.grad.cpu().numpy().copy() for k, p in m.named_parameters()}))
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


def test_two_rank_dropout_masks_are_global_batch_masks():
    """With dropout on, rank r's rows draw the masks of global rows r*B_l.. (mask row
    offset rank * B_l * T, tt_gru_fwd_rec.drop_row0): the two ranks never repeat each
    other's masks, and their outputs and summed gradients equal the single-process
    train-mode step on the whole batch with the same seeds."""
    import numpy as np

    import two_towers_amd as tta
    z = _dp_golden()
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_drop_rank, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = out.get(timeout=120)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m = _dp_model(z).train()
    torch.manual_seed(40)
    qv, dv = m(torch.from_numpy(z["q"]).cuda(), torch.from_numpy(z["d"]).cuda())
    tta.InfoNCELoss()(qv, dv).backward()
    q1 = qv.detach().cpu().numpy()
    n = q1.shape[0] // 2
    for r in range(2):
        np.testing.assert_allclose(res[r][0], q1[r * n:(r + 1) * n], rtol=0, atol=1e-5 * np.abs(q1).max())
    for k, p in m.named_parameters():
        g = p.grad.cpu().numpy()
        for r in range(2):
            assert float(np.abs(res[r][1][k] - g).max()) <= 1e-4 * float(np.abs(g).max()) + 1e-9, (r, k)
    # the eval outputs differ from the train outputs: dropout really ran
    with torch.no_grad():
        qe, _ = m.eval()(torch.from_numpy(z["q"]).cuda(), torch.from_numpy(z["d"]).cuda())
    assert float((qe.cpu() - torch.from_numpy(q1)).abs().max()) > 1e-4


def _bench_scale_rank(port, use_pg, out):
    """One bench-composition step at bench scale (E 300, h 256, T 64, bf16, dropout 0.1,
    B 1024, hard-negative margin loss, Adam) with the column-split GRU forward, either
    plain or inside a one-rank RCCL process group with every collective forced on."""
    import numpy as np
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if use_pg:
        os.environ["TT_DIST_FORCE"] = "1"
        torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import two_towers_amd as tta
        from two_towers_amd import _lib
        from two_towers_amd import dist as tdp
        _lib.set_option("gru_fwd_xc", 1)
        torch.manual_seed(5)
        m = tta.EnhancedTwoTowerModel(300, 256).cuda().set_compute_dtype(torch.bfloat16).train()
        m.set_process_group(None, overlap_grad_allreduce=True)
        assert _lib.load().tt_gru_fwd_ws_size(_lib.DT_BF16, 4, 1024, 64, 512, 3072, 1024) > 0, "xcp expected"
        g = torch.Generator().manual_seed(6)
        q = (torch.randn(1024, 64, 300, generator=g) * 0.5).cuda()
        d = (torch.randn(1024, 64, 300, generator=g) * 0.5).cuda()
        crit = tta.HardNegativeMarginLoss(k=5, margin=0.2, compute_dtype=torch.bfloat16)
        opt = tta.Adam(m.parameters(), lr=1e-3)
        torch.manual_seed(7)
        loss = crit(*m(q, d))
        loss.backward()
        tdp.allreduce_grads(list(m.parameters()))
        opt.step()
        tta.check_gru_status()
        out.put((float(loss.detach()), {k: v.detach().cpu().float().numpy().copy() for k, v in m.state_dict().items()},
                 crit.last_indices.cpu().numpy().copy(),
                 {k: p.grad.detach().cpu().float().numpy().copy() for k, p in m.named_parameters()}))
    finally:
        if use_pg:
            torch.distributed.destroy_process_group()


def test_rccl_one_rank_bench_scale_step_is_bit_identical():
    """The bench's kernels under a process group: the column-split forward, the streamed
    hard-negative scan, the overlapped gradient all-reduce on RCCL's stream. With one rank
    every collective is an identity, so the loss, the mined indices and every weight after
    Adam must be bit-identical to the same step without a process group."""
    import numpy as np
    ctx = mp.get_context("spawn")
    res = []
    for use_pg in (False, True):
        out = ctx.Queue()
        p = ctx.Process(target=_bench_scale_rank, args=(_port(), use_pg, out))
        p.start()
        res.append(out.get(timeout=240))
        p.join(timeout=60)
        assert p.exitcode == 0
    (l0, w0, i0, g0), (l1, w1, i1, g1) = res
    assert l0 == l1, (l0, l1)
    assert (i0 == i1).all()
    assert set(w0) == set(w1) and len(g0) == 44 and set(g0) == set(g1)
    for k in w0:  # both towers: every kernel of the step is deterministic
        assert np.array_equal(w0[k], w1[k]), k
    for k in g0:
        assert np.array_equal(g0[k], g1[k]), k
