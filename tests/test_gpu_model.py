"""Model-level parity on the GPU against the CPU oracle (oracle/cpu_ref.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import two_towers_amd as tta  # noqa: E402
from oracle import cpu_ref  # noqa: E402
from two_towers_amd._lib import option  # noqa: E402

DEV = "cuda"


def make_model(E, h, seed=0):
    torch.manual_seed(seed)
    m = tta.EnhancedTwoTowerModel(E, h)
    p = {k: v.detach().clone() for k, v in m.state_dict().items()}
    return m, p


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("E,h,B,T", [(16, 8, 16, 8), (40, 32, 100, 12), (300, 64, 64, 16)])
def test_forward_backward_fp32(E, h, B, T):
    m, p = make_model(E, h)
    m = m.to(DEV).eval()
    g = torch.Generator().manual_seed(5)
    q = torch.randn(B, T, E, generator=g)
    d = torch.randn(B, T, E, generator=g)
    qv, dv = m(q.to(DEV), d.to(DEV))
    loss = tta.InfoNCELoss()(qv, dv)
    loss.backward()
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    rq, rd = cpu_ref.forward(q, d, pr)
    rl = cpu_ref.infonce(rq, rd)
    rl.backward()
    assert rel(qv, rq) < 1e-4 and rel(dv, rd) < 1e-4
    assert abs(float(loss) - float(rl)) < 1e-4 * max(1.0, abs(float(rl)))
    named = dict(m.named_parameters())
    worst = max(rel(named[k].grad, pr[k].grad) for k in pr)
    assert worst < 2e-3, {k: rel(named[k].grad, pr[k].grad) for k in pr}


def test_forward_backward_bf16():
    """bf16 storage / fp32 accumulation vs the fp32 oracle run on the same bf16-rounded
    inputs and weights (so only the kernels' internal rounding is compared).
    Tolerances: loss 1e-3 relative; per-parameter gradient cos >= 0.998 and
    ||g - g_ref|| <= 6% ||g_ref||."""
    E, h, B, T = 64, 32, 96, 10
    m, _ = make_model(E, h, 1)
    with torch.no_grad():
        for prm in m.parameters():
            prm.copy_(prm.to(torch.bfloat16).float())
    p = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV).eval().set_compute_dtype(torch.bfloat16)
    g = torch.Generator().manual_seed(6)
    q = torch.randn(B, T, E, generator=g).to(torch.bfloat16).float()
    d = torch.randn(B, T, E, generator=g).to(torch.bfloat16).float()
    qv, dv = m(q.to(DEV), d.to(DEV))
    loss = tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv)
    loss.backward()
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    rq, rd = cpu_ref.forward(q, d, pr)
    rl = cpu_ref.infonce(rq, rd)
    rl.backward()
    assert rel(qv, rq) < 3e-2 and rel(dv, rd) < 3e-2
    assert abs(float(loss) - float(rl)) < 1e-3 * abs(float(rl))
    named = dict(m.named_parameters())
    for k in pr:
        a, b = named[k].grad.double().cpu(), pr[k].grad.double()
        cos = float((a * b).sum() / (a.norm() * b.norm()))
        frob = float((a - b).norm() / b.norm())
        assert cos >= 0.998 and frob <= 0.06, (k, cos, frob)


def test_dropout_matches_counter_mask():
    E, h, B, T = 24, 16, 40, 6
    m, p = make_model(E, h, 2)
    m = m.to(DEV).train()
    g = torch.Generator().manual_seed(7)
    q = torch.randn(B, T, E, generator=g)
    torch.manual_seed(99)
    qv = m.encode_query(q.to(DEV))
    torch.manual_seed(99)
    seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
    rq = cpu_ref.encode(q, p, "query", drop_p=0.1, seed=seed)
    assert rel(qv, rq) < 1e-4


def test_margin_hardneg_fp32():
    B, h = 64, 16
    g = torch.Generator().manual_seed(8)
    q = torch.randn(B, h, generator=g)
    d = torch.randn(B, h, generator=g)
    qd, dd = q.clone().to(DEV).requires_grad_(True), d.clone().to(DEV).requires_grad_(True)
    lossf = tta.HardNegativeMarginLoss(k=5, margin=0.2)
    loss = lossf(qd, dd)
    loss.backward()
    qr, dr = q.clone().requires_grad_(True), d.clone().requires_grad_(True)
    rl, ridx = cpu_ref.hardneg_margin(qr, dr, 5, 0.2)
    rl.backward()
    assert torch.equal(lossf.last_indices.long().cpu(), ridx)
    assert abs(float(loss) - float(rl)) < 1e-5
    assert rel(qd.grad, qr.grad) < 1e-4 and rel(dd.grad, dr.grad) < 1e-4


def test_margin_inbatch_and_explicit():
    B, h, k = 32, 24, 3
    g = torch.Generator().manual_seed(9)
    q, d, n = torch.randn(B, h, generator=g), torch.randn(B, h, generator=g), torch.randn(B * k, h, generator=g)
    for neg in (None, n):
        ts = [t.clone().to(DEV).requires_grad_(True) for t in (q, d)] + ([n.clone().to(DEV).requires_grad_(True)] if neg is not None else [])
        rs = [t.clone().requires_grad_(True) for t in (q, d)] + ([n.clone().requires_grad_(True)] if neg is not None else [])
        l1 = tta.MarginRankingLoss()(*ts)
        l2 = cpu_ref.margin_loss(*rs)
        l1.backward()
        l2.backward()
        assert abs(float(l1) - float(l2)) < 1e-4 * max(1, abs(float(l2)))
        for a, b in zip(ts, rs):
            assert rel(a.grad, b.grad) < 1e-4


def test_get_hard_negatives_single():
    g = torch.Generator().manual_seed(10)
    q = torch.randn(32, generator=g)
    docs = torch.randn(500, 32, generator=g)
    idx = tta.get_hard_negatives(q.to(DEV), docs.to(DEV), 17, k=5)
    assert torch.equal(idx.cpu(), cpu_ref.hard_negatives(q, docs, 17, 5))


def test_token_ids_match_float_inputs():
    E, h, B, T, V = 32, 16, 20, 9, 50
    m, p = make_model(E, h, 3)
    m = m.to(DEV).eval()
    table = torch.randn(V, E)
    ids = torch.randint(-1, V, (B, T), dtype=torch.int32)
    emb = torch.where((ids >= 0)[..., None], table[ids.clamp_min(0).long()], torch.zeros(E))
    m.set_embedding_table(table.to(DEV))
    a = m.encode_doc(ids.to(DEV))
    b = m.encode_doc(emb.to(DEV))
    assert torch.allclose(a, b, rtol=0, atol=0)


def test_cpu_tensors_fail_loudly():
    m, _ = make_model(16, 8)
    with pytest.raises(RuntimeError, match="GPU"):
        m(torch.randn(2, 3, 16), torch.randn(2, 3, 16))


@pytest.mark.parametrize("h,B,T", [(32, 96, 10), (64, 200, 7), (128, 70, 4), (256, 130, 5)])
def test_persistent_gru_matches_step_kernel(h, B, T):
    """bf16 forward + backward through the persistent (row-resident) GRU forward
    kernel vs the per-step kernel (option gru_step = 1): same arithmetic in the same
    order, so outputs and gradients are bit-identical. h 32 / 64 (H 64 / 128) run the
    runtime-width instances restored after the store-hazard fix."""
    E = 48
    g = torch.Generator().manual_seed(11)
    q = torch.randn(B, T, E, generator=g).to(DEV)
    d = torch.randn(B, T, E, generator=g).to(DEV)
    outs = []
    for step in (1, 0):
        m, _ = make_model(E, h, 3)
        m = m.to(DEV).train().set_compute_dtype(torch.bfloat16)
        with option("gru_step", step):
            qv, dv = m(q, d)
            loss = tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv)
            loss.backward()
        outs.append((qv.detach().clone(), dv.detach().clone(), {k: p.grad.clone() for k, p in m.named_parameters()}))
    (q0, d0, g0), (q1, d1, g1) = outs
    assert torch.equal(q1, q0) and torch.equal(d1, d0)
    for k in g0:
        assert torch.equal(g1[k], g0[k]), (k, rel(g1[k], g0[k]))


def test_training_step_is_deterministic():
    """Two identical bf16 train-mode forward + InfoNCE + backward passes give bit-identical
    outputs and all 44 gradients: no float atomics on the path (bias and LayerNorm sums
    run in a fixed order, split-K and the fused InfoNCE backward reduce fp32 slabs).
    (HardNegativeMarginLoss is the exception: its document-gradient scatter adds repeated
    negatives with float atomics, so the doc tower's gradients may differ in the last bit;
    DESIGN.md §4.)"""
    E, h, B, T = 48, 64, 300, 7
    g = torch.Generator().manual_seed(17)
    q = torch.randn(B, T, E, generator=g).to(DEV)
    d = torch.randn(B, T, E, generator=g).to(DEV)
    outs = []
    for _ in range(2):
        m, _ = make_model(E, h, 4)
        m = m.to(DEV).train().set_compute_dtype(torch.bfloat16)
        torch.manual_seed(6)
        qv, dv = m(q, d)
        tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv).backward()
        outs.append((qv.detach().clone(), dv.detach().clone(), {k: p.grad.clone() for k, p in m.named_parameters()}))
    (q0, d0, g0), (q1, d1, g1) = outs
    assert torch.equal(q1, q0) and torch.equal(d1, d0)
    for k in g0:
        assert torch.equal(g1[k], g0[k]), k


@pytest.mark.parametrize("B,T", [(130, 5), (520, 3)])
def test_big_tile_gru_backward_matches_step_kernel(B, T):
    """bf16 H=512 backward on 256x256 tiles (8-phase GEMM, two-pass epilogue) vs the
    128x128 step kernels (option gru_bwd_big = 0): gradients agree to accumulation order."""
    E, h = 40, 256
    g = torch.Generator().manual_seed(12)
    q = torch.randn(B, T, E, generator=g).to(DEV)
    d = torch.randn(B, T, E, generator=g).to(DEV)
    outs = []
    for big in (0, 1):
        m, _ = make_model(E, h, 4)
        m = m.to(DEV).train().set_compute_dtype(torch.bfloat16)
        with option("gru_bwd_big", big):
            qv, dv = m(q, d)
            loss = tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv)
            loss.backward()
        outs.append({k: p.grad.clone() for k, p in m.named_parameters()})
    for k in outs[0]:
        a, b = outs[1][k].double(), outs[0][k].double()
        cos = float((a * b).sum() / (a.norm() * b.norm() + 1e-30))
        assert cos > 0.9999 and rel(outs[1][k], outs[0][k]) < 2e-2, (k, cos)


@pytest.mark.parametrize("h,B,T", [(256, 130, 5), (256, 520, 3), (128, 200, 6), (512, 300, 4), (512, 130, 3)])
def test_row_owning_gru_backward_matches_step_kernels(h, B, T):
    """bf16 backward through the persistent row-owning kernel (one launch per layer,
    H 1024 / 512 / 256: gru_bwd_rows, 128 rows x all H units per workgroup; H 1024 in two
    column passes of 512 units per step) vs the
    per-step launches (option gru_bwd_persist = 0): the same arithmetic per element, so
    gradients agree to accumulation order (the recurrent GEMM's K order and the bias
    partial sums differ). B 130 / 520 / 200 give tail row tiles."""
    E = 40
    g = torch.Generator().manual_seed(13)
    q = torch.randn(B, T, E, generator=g).to(DEV)
    d = torch.randn(B, T, E, generator=g).to(DEV)
    outs = []
    for persist in (0, 1):
        m, _ = make_model(E, h, 5)
        m = m.to(DEV).train().set_compute_dtype(torch.bfloat16)
        with option("gru_bwd_persist", 2 * persist):  # 2: the row-owning kernel at H 1024 too
            qv, dv = m(q, d)
            loss = tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv)
            loss.backward()
        outs.append({k: p.grad.clone() for k, p in m.named_parameters()})
    for k in outs[0]:
        a, b = outs[1][k].double(), outs[0][k].double()
        cos = float((a * b).sum() / (a.norm() * b.norm() + 1e-30))
        assert cos > 0.9999 and rel(outs[1][k], outs[0][k]) < 2e-2, (k, cos)


def test_packed_weight_cache_follows_parameter_versions():
    """Inference calls reuse the packed compute copies of the weights (towers._packed)
    while the parameters are unchanged, and repack after an optimizer step
    (two_towers_amd.Adam bumps the versions) or load_state_dict: outputs always equal a
    freshly built model holding the same weights."""
    E, h, B, T = 32, 16, 40, 6
    m, _ = make_model(E, h, 21)
    m = m.to(DEV).set_compute_dtype(torch.bfloat16)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, T, E, generator=g).to(DEV)
    y = torch.randn(B, T, E, generator=g).to(DEV)
    p0 = m.query_encoder.weight_ih_l0

    def fresh_out():
        f, _ = make_model(E, h, 0)
        f.load_state_dict(m.state_dict())
        f = f.to(DEV).set_compute_dtype(torch.bfloat16).eval()
        with torch.no_grad():
            return f.encode_query(x)

    m.eval()
    with torch.no_grad():
        a = m.encode_query(x)
        pk = p0._tt_pack[1]
        b = m.encode_query(x)
    assert p0._tt_pack[1] is pk and torch.equal(a, b)
    m.train()
    opt = tta.Adam(m.parameters(), lr=1e-2)
    qv, dv = m(x, y)
    tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv).backward()
    opt.step()
    m.eval()
    with torch.no_grad():
        c = m.encode_query(x)
    assert p0._tt_pack[1] is not pk and not torch.equal(c, a)
    assert torch.equal(c, fresh_out())
    sd = {k: v + 0.01 for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    with torch.no_grad():
        d = m.encode_query(x)
    assert torch.equal(d, fresh_out())


@pytest.mark.parametrize("h,B,T,dt", [(512, 300, 3, torch.bfloat16), (48, 520, 4, torch.float32)])
def test_per_step_forward_256_row_tiles(h, B, T, dt):
    """Per-step GRU forward (the path of H > 512 in bf16, e.g. configs[4]'s H = 1024, and of
    fp32) on 256-row tiles (8 waves) vs 128-row tiles (option gru_fwd_step_rows): the same
    K order per output, so outputs and gradients agree to fp32 rounding. B 300 / 520 give
    tail row tiles."""
    E = 40
    g = torch.Generator().manual_seed(15)
    q = torch.randn(B, T, E, generator=g).to(DEV)
    d = torch.randn(B, T, E, generator=g).to(DEV)
    outs = []
    for rows in (128, 256):
        m, _ = make_model(E, h, 3)
        m = m.to(DEV).train().set_compute_dtype(dt)
        with option("gru_step", 1), option("gru_fwd_step_rows", rows):
            qv, dv = m(q, d)
            loss = tta.InfoNCELoss(compute_dtype=dt)(qv, dv)
            loss.backward()
        outs.append((qv.detach().clone(), dv.detach().clone(), {k: p.grad.clone() for k, p in m.named_parameters()}))
    q0, d0, g0 = outs[0]
    for q1, d1, g1 in outs[1:]:
        assert rel(q1, q0) < 1e-5 and rel(d1, d0) < 1e-5
        for k in g0:
            assert rel(g1[k], g0[k]) < 1e-4, k


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,T", [(1, 1), (1, 30), (2, 1), (3, 64)])
def test_tiny_batches_and_sequences(B, T, dt):
    """Edge shapes of the drop-in surface: validate_enhanced.py:61-71 encodes ONE text at a
    time ([1, T, E]), T = 1 has no recurrent term past the first step, B = 2 / 3 leave
    almost every row tile empty. encode_query / encode_doc and a train-mode InfoNCE
    backward against the oracle (fp32: 1e-4 outputs, 2e-3 gradients; bf16: the operand
    rounding of the bench-path tests, 3e-2 outputs)."""
    E, h = 300, 64
    m, p = make_model(E, h, 17)
    m = m.to(DEV).set_compute_dtype(dt).eval()
    g = torch.Generator().manual_seed(B * 100 + T)
    q = torch.randn(B, T, E, generator=g) * 0.5
    d = torch.randn(B, T, E, generator=g) * 0.5
    if dt == torch.bfloat16:
        q, d = q.to(dt).float(), d.to(dt).float()
        p = {k: v.to(dt).float() for k, v in p.items()}
        m.load_state_dict(p)
    tol = 1e-4 if dt == torch.float32 else 3e-2
    with torch.no_grad():
        eq = m.encode_query(q.to(DEV))
        ed = m.encode_doc(d.to(DEV))
    assert eq.shape == (B, h) and ed.shape == (B, h)
    assert rel(eq, cpu_ref.encode(q, p, "query")) < tol and rel(ed, cpu_ref.encode(d, p, "doc")) < tol
    if B < 2:
        return
    qv, dv = m(q.to(DEV), d.to(DEV))
    loss = tta.InfoNCELoss(compute_dtype=dt)(qv, dv)
    loss.backward()
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    rl = cpu_ref.infonce(*cpu_ref.forward(q, d, pr))
    rl.backward()
    lv, rv = float(loss.detach()), float(rl.detach())
    assert abs(lv - rv) < (1e-4 if dt == torch.float32 else 2e-2) * max(1.0, abs(rv))
    if dt == torch.float32:
        named = dict(m.named_parameters())
        worst = max(rel(named[k].grad, pr[k].grad) for k in pr)
        assert worst < 2e-3, worst
