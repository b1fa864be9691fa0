"""Parity of the configuration bench.py measures against the fp32 CPU oracle.

BASELINE configs[2] runs EnhancedTwoTowerModel(300, 256) (GRU H = 512 per direction),
seq_len 64, bf16, dropout 0.1, hard-negative mining k = 5 + MarginRankingLoss(0.2).
These tests run the kernels that step runs -- the column-split persistent GRU forward
(gru_fwd_xs<512, *>, which bench.py's B 8192 selects; forced here with option
gru_fwd_xc = 2 because its auto mode needs B >= 1024 and the oracle wants a small batch)
and the row-owning one it falls back to (gru_fwd_seq<4, 8>, the auto choice at these
batches), the row-owning BPTT kernel (gru_bwd_rows<512>, one launch per layer), the
persistent input-projection GEMMs, the fp32 head, the hard-negative scan -- at a batch
the oracle finishes in seconds, and
compare with oracle/cpu_ref.py (reference enhanced_two_tower.py:50-65, :67-82, :84-133)
evaluated in fp32 on the same bf16-rounded weights and inputs, so only the kernels'
internal bf16 rounding (operands of every MFMA, the saved pre-activations, the bf16
BPTT carry over 64 steps) is measured.

Tolerances, stated here and asserted below:
  * loss: relative error <= 2e-3;
  * tower outputs: max-abs error <= 3e-2 of the largest entry;
  * every 2-D weight gradient (28 of the 44): cosine similarity >= 0.998 and
    ||g - g_ref|| <= 0.06 ||g_ref||;
  * every 1-D gradient (GRU biases, head biases, LayerNorm affine; 16 of the 44):
    cosine >= 0.996 and ||g - g_ref|| <= 0.09 ||g_ref||. These are column sums over
    B*T = 16,384 (GRU) or B rows whose terms largely cancel, so the 2^-9 relative
    rounding of the bf16-stored gate inputs, pre-activations and gate gradients shows
    up amplified in the small residual. Measured worst case over two weight seeds x
    dropout off/on (tools/diag_bench_path.py): cos 0.9977, 6.7 % (a bias of the layer-0
    reverse recurrence); weights <= 5.5 %. An fp32 BPTT carry changed none of these
    numbers: the carry is not the error source;
  * hard negatives in bf16 vs the fp32 oracle at B = 1024: >= 97 % of the rows pick the
    same set of k indices, every differing pick is a near-tie (its fp32 cosine within
    4e-3 of the oracle's k-th best), and the loss on the picked indices equals the fp32
    margin loss on those indices to 1e-5.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import two_towers_amd as tta  # noqa: E402
from oracle import cpu_ref  # noqa: E402
from two_towers_amd import _lib  # noqa: E402
from two_towers_amd._lib import option  # noqa: E402

DEV = "cuda"
E, HID, T, B = 300, 256, 64, 256  # GRU H = 2 * HID = 512


def _bf16(x):
    return x.to(torch.bfloat16).float()


def _model(seed):
    torch.manual_seed(seed)
    m = tta.EnhancedTwoTowerModel(E, HID)
    with torch.no_grad():
        for prm in m.parameters():
            prm.copy_(_bf16(prm))
    p = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    return m.to(DEV).set_compute_dtype(torch.bfloat16), p


def _grad_check(named, ref):
    worst = []
    for k, pr in ref.items():
        a, b = named[k].grad.double().cpu(), pr.grad.double()
        cos = float((a * b).sum() / (a.norm() * b.norm() + 1e-300))
        frob = float((a - b).norm() / (b.norm() + 1e-300))
        worst.append((frob, cos, k))
        cmin, rmax = (0.998, 0.06) if b.dim() == 2 else (0.996, 0.09)
        assert cos >= cmin and frob <= rmax, (k, cos, frob)
    return max(worst)


def _xc_forced(xc):
    """option gru_fwd_xc: 1 = auto (row-owning gru_fwd_seq at these batches), 2 = the
    column-split gru_fwd_xs forced; asserts which one the shape gets."""
    lib = _lib.load()
    ws = lib.tt_gru_fwd_ws_size(_lib.DT_BF16, 4, B, T, 2 * HID, 6 * 2 * HID, 2 * 2 * HID)
    assert (ws > 0) == (xc == 2), (xc, ws)
    assert lib.tt_gru_fwd_launches(_lib.DT_BF16, T, 2 * HID) == 1, "persistent forward expected at H=512"


@pytest.mark.parametrize("xc", [1, 2])
@pytest.mark.parametrize("drop_p", [0.0, 0.1])
def test_bench_config_bf16_matches_oracle(drop_p, xc):
    m, p = _model(31)
    m.train() if drop_p > 0 else m.eval()
    g = torch.Generator().manual_seed(32)
    q = _bf16(torch.randn(B, T, E, generator=g) * 0.5)
    d = _bf16(torch.randn(B, T, E, generator=g) * 0.5)
    torch.manual_seed(33)  # the forward draws one dropout seed per tower from this stream
    with option("gru_fwd_xc", xc):
        _xc_forced(xc)
        qv, dv = m(q.to(DEV), d.to(DEV))
        loss = tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv)
        loss.backward()
    tta.check_gru_status()
    torch.manual_seed(33)
    seeds = [int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) for _ in range(2)] if drop_p > 0 else [0, 0]
    rq, rd = cpu_ref.forward(q, d, p, drop_p=drop_p, seeds=seeds)
    rl = cpu_ref.infonce(rq, rd)
    rl.backward()
    lv, rv = float(loss.detach()), float(rl.detach())
    assert abs(lv - rv) <= 2e-3 * abs(rv), (lv, rv)
    for a, b in ((qv, rq), (dv, rd)):
        a, b = a.detach().double().cpu(), b.detach().double()
        assert float((a - b).abs().max() / b.abs().max()) <= 3e-2
    frob, cos, k = _grad_check(dict(m.named_parameters()), p)
    print(f"drop {drop_p}: loss {lv:.6f} vs {rv:.6f}; worst gradient {k}: rel {frob:.4f}, cos {cos:.5f}")


def test_hardneg_margin_bf16_b1024_agrees_with_fp32():
    Bq, h, k = 1024, 256, 5
    g = torch.Generator().manual_seed(34)
    d = torch.randn(Bq, h, generator=g)
    q = d + 4.0 * torch.randn(Bq, h, generator=g)  # pos cos ~0.24, top negatives ~0.2: hinges active
    qd, dd = q.clone().to(DEV).requires_grad_(True), d.clone().to(DEV).requires_grad_(True)
    crit = tta.HardNegativeMarginLoss(k=k, margin=0.2, compute_dtype=torch.bfloat16)
    loss = crit(qd, dd)
    loss.backward()
    idx = crit.last_indices.long().cpu()
    _, ridx = cpu_ref.hardneg_margin(q.clone(), d.clone(), k, 0.2)
    same = np.array([set(idx[i].tolist()) == set(ridx[i].tolist()) for i in range(Bq)])
    assert same.mean() >= 0.97, same.mean()
    # every disagreement is a near-tie of the fp32 ranking
    cos = cpu_ref.normalize(q, 1e-8) @ cpu_ref.normalize(d, 1e-8).t()
    cos.fill_diagonal_(-1.0)
    kth = cos.gather(1, ridx)[:, -1]
    for i in np.nonzero(~same)[0]:
        for j in set(idx[i].tolist()) - set(ridx[i].tolist()):
            assert float(kth[i] - cos[i, j]) <= 4e-3, (i, j, float(kth[i]), float(cos[i, j]))
    # given the picked indices, the loss and its gradients are the fp32 margin loss
    qr, dr = q.clone().requires_grad_(True), d.clone().requires_grad_(True)
    rl = cpu_ref.margin_loss(qr, dr, dr[idx.reshape(-1)], 0.2)
    rl.backward()
    assert float(rl.detach()) > 0.01, "hinges inactive: the test would compare zeros"
    assert abs(float(loss.detach()) - float(rl.detach())) <= 1e-5
    for a, b in ((qd.grad, qr.grad), (dd.grad, dr.grad)):
        a, b = a.double().cpu(), b.double()
        assert float((a - b).abs().max() / b.abs().max()) <= 1e-4
    print(f"hard negatives: {same.mean():.4f} of rows pick the fp32 set; loss {float(loss):.6f}")


def test_reference_size_h512_bf16_matches_oracle():
    """hidden_dim 512 (GRU H = 1024), the reference's own training size
    (train_enhanced.py:30) and BASELINE configs[4]'s model, in bf16 at T = 32 (configs[4]
    runs T = 128): the per-step bf16 forward (H > 512 exceeds the row-resident kernel's
    LDS image) and the 256x256 BPTT step kernel (gru_bwd_big), against the fp32 oracle on
    bf16-rounded operands, with the tolerances stated at the top of this file."""
    Hd, Tq, Bq = 512, 32, 64
    torch.manual_seed(35)
    m = tta.EnhancedTwoTowerModel(E, Hd)
    with torch.no_grad():
        for prm in m.parameters():
            prm.copy_(_bf16(prm))
    p = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    m = m.to(DEV).set_compute_dtype(torch.bfloat16).train()
    g = torch.Generator().manual_seed(36)
    q = _bf16(torch.randn(Bq, Tq, E, generator=g) * 0.5)
    d = _bf16(torch.randn(Bq, Tq, E, generator=g) * 0.5)
    torch.manual_seed(37)
    qv, dv = m(q.to(DEV), d.to(DEV))
    loss = tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv)
    loss.backward()
    torch.manual_seed(37)
    seeds = [int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) for _ in range(2)]
    rq, rd = cpu_ref.forward(q, d, p, drop_p=0.1, seeds=seeds)
    rl = cpu_ref.infonce(rq, rd)
    rl.backward()
    lv, rv = float(loss.detach()), float(rl.detach())
    assert abs(lv - rv) <= 2e-3 * abs(rv), (lv, rv)
    for a, b in ((qv, rq), (dv, rd)):
        a, b = a.detach().double().cpu(), b.detach().double()
        assert float((a - b).abs().max() / b.abs().max()) <= 3e-2
    frob, cos, k = _grad_check(dict(m.named_parameters()), p)
    print(f"h 512: loss {lv:.6f} vs {rv:.6f}; worst gradient {k}: rel {frob:.4f}, cos {cos:.5f}")


@pytest.mark.parametrize("xc", [1, 2])
def test_bench_composition_hardneg_margin_matches_oracle(xc):
    """The step bench.py times, end to end at B = 512: EnhancedTwoTowerModel(300, 256),
    T 64, bf16, dropout 0.1, HardNegativeMarginLoss (get_hard_negatives k = 5 over the
    in-batch documents + MarginRankingLoss(0.2) on the gathered rows,
    enhanced_two_tower.py:84-133 as composed in SURVEY.md §3.3) and the backward, against
    cpu_ref.forward + cpu_ref.hardneg_margin in fp32 on the same bf16-rounded operands and
    dropout masks.

    Mining: the GPU mines on its bf16 tower outputs, the oracle on its fp32 ones, which
    differ by up to 3e-2 of the largest entry; so >= 90 % of the rows must pick the
    oracle's set and every other pick must be a near-tie, its oracle cosine within 2e-2 of
    the oracle's k-th best. Loss and gradients: given the GPU's picks, the oracle's margin
    loss through the oracle's forward/backward (so a differing near-tie pick is not counted
    as a gradient error): loss relative 5e-3, tower outputs as above, gradients with the
    tolerances stated at the top of this file. xc 2: with the column-split forward bench.py
    runs at B 8192 (gru_fwd_xs), forced at this batch. The same step with nothing forced (B
    1024): test_bench_b1024_unforced_kernel_selection_matches_oracle."""
    Bq, k = 512, 5
    m, p = _model(41)
    m.train()
    g = torch.Generator().manual_seed(42)
    q = _bf16(torch.randn(Bq, T, E, generator=g) * 0.5)
    d = _bf16(torch.randn(Bq, T, E, generator=g) * 0.5)
    crit = tta.HardNegativeMarginLoss(k=k, margin=0.2, compute_dtype=torch.bfloat16)
    torch.manual_seed(43)
    with option("gru_fwd_xc", xc):
        lib = _lib.load()
        assert (lib.tt_gru_fwd_ws_size(_lib.DT_BF16, 4, Bq, T, 2 * HID, 6 * 2 * HID, 2 * 2 * HID) > 0) == (xc == 2)
        qv, dv = m(q.to(DEV), d.to(DEV))
        loss = crit(qv, dv)
        loss.backward()
    tta.check_gru_status()
    idx = crit.last_indices.long().cpu()
    torch.manual_seed(43)
    seeds = [int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) for _ in range(2)]
    rq, rd = cpu_ref.forward(q, d, p, drop_p=0.1, seeds=seeds)
    with torch.no_grad():
        _, ridx = cpu_ref.hardneg_margin(rq.detach(), rd.detach(), k, 0.2)
        cos = cpu_ref.normalize(rq.detach(), 1e-8) @ cpu_ref.normalize(rd.detach(), 1e-8).t()
        cos.fill_diagonal_(-1.0)
        kth = cos.gather(1, ridx)[:, -1]
    same = np.array([set(idx[i].tolist()) == set(ridx[i].tolist()) for i in range(Bq)])
    worst = 0.0
    for i in np.nonzero(~same)[0]:
        for j in set(idx[i].tolist()) - set(ridx[i].tolist()):
            worst = max(worst, float(kth[i] - cos[i, j]))
    print(f"composition: {same.mean():.4f} of rows pick the fp32 set, worst near-tie gap {worst:.2e}")
    assert same.mean() >= 0.90, same.mean()
    assert worst <= 2e-2, worst
    rl = cpu_ref.margin_loss(rq, rd, rd[idx.reshape(-1)], 0.2)
    rl.backward()
    lv, rv = float(loss.detach()), float(rl.detach())
    assert rv > 0.01, "hinges inactive: the test would compare zeros"
    assert abs(lv - rv) <= 5e-3 * abs(rv), (lv, rv)
    for a, b in ((qv, rq), (dv, rd)):
        a, b = a.detach().double().cpu(), b.detach().double()
        assert float((a - b).abs().max() / b.abs().max()) <= 3e-2
    frob, c, kname = _grad_check(dict(m.named_parameters()), p)
    print(f"composition: loss {lv:.6f} vs {rv:.6f}; worst gradient {kname}: rel {frob:.4f}, cos {c:.5f}")


def test_reference_size_h512_t128_bf16_matches_oracle():
    """configs[4]'s model and sequence length: hidden_dim 512 (GRU H = 1024,
    train_enhanced.py:30, enhanced_two_tower.py:19), T = 128, bf16, dropout 0.1, B = 16,
    InfoNCE + backward, against the fp32 oracle on bf16-rounded operands. Runs the kernels
    configs[4] runs (per-step bf16 forward, 256 x 256 per-step BPTT) over 128 steps, so the
    bf16 rounding of the recurrent state, the saved pre-activations and the BPTT carry
    compounds over twice the steps of the bench configuration; tolerances as stated at the
    top of this file."""
    Hd, Tq, Bq = 512, 128, 16
    torch.manual_seed(38)
    m = tta.EnhancedTwoTowerModel(E, Hd)
    with torch.no_grad():
        for prm in m.parameters():
            prm.copy_(_bf16(prm))
    p = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    m = m.to(DEV).set_compute_dtype(torch.bfloat16).train()
    g = torch.Generator().manual_seed(39)
    q = _bf16(torch.randn(Bq, Tq, E, generator=g) * 0.5)
    d = _bf16(torch.randn(Bq, Tq, E, generator=g) * 0.5)
    torch.manual_seed(40)
    qv, dv = m(q.to(DEV), d.to(DEV))
    loss = tta.InfoNCELoss(compute_dtype=torch.bfloat16)(qv, dv)
    loss.backward()
    torch.manual_seed(40)
    seeds = [int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) for _ in range(2)]
    rq, rd = cpu_ref.forward(q, d, p, drop_p=0.1, seeds=seeds)
    rl = cpu_ref.infonce(rq, rd)
    rl.backward()
    lv, rv = float(loss.detach()), float(rl.detach())
    assert abs(lv - rv) <= 2e-3 * abs(rv), (lv, rv)
    for a, b in ((qv, rq), (dv, rd)):
        a, b = a.detach().double().cpu(), b.detach().double()
        assert float((a - b).abs().max() / b.abs().max()) <= 3e-2
    frob, cos, k = _grad_check(dict(m.named_parameters()), p)
    print(f"h 512 T 128: loss {lv:.6f} vs {rv:.6f}; worst gradient {k}: rel {frob:.4f}, cos {cos:.5f}")


def test_bench_b1024_unforced_kernel_selection_matches_oracle():
    """One training step of the bench composition at B 1024, T 64 (M = B*T = 65,536 GEMM
    rows) with every option at its default, so the GPU runs bench.py's own kernel selection
    UNFORCED -- the column-split GRU forward (gru_fwd_xs, auto from B 1024), the B-resident
    layer-0 projection (gemm_bres), the persistent layer-1 projection (gemm_persist), the
    split-K weight gradients, the row-owning BPTT and the hard-negative scan -- against the
    fp32 oracle's step on the same bf16-rounded weights, correlated inputs and dropout masks
    (tests/golden/bench_b1024.npz, oracle/gen_b1024.py; ~2 minutes of CPU, so computed once).
    (enhanced_two_tower.py:50-65, :84-133; train_enhanced.py:58-62.)

    Tolerances: >= 90 % of the rows mine the oracle's set and every other pick is a near-tie,
    its oracle cosine within 1e-2 of the oracle's k-th best (the GPU mines on its bf16 tower
    outputs); loss relative 5e-3; tower outputs (128 sampled rows) max-abs 3e-2 of the largest
    entry. Gradients: the step's backward is run a second time with the ORACLE's negatives
    through HardNegativeMarginLoss's own margin step (same kernels), so a near-tie
    picked differently is not counted as a gradient error; on 16,384 fixed positions per
    tensor (all of the smaller ones): the 2-D / 1-D cosine and relative-Frobenius bounds
    stated at the top of this file."""
    import os
    from oracle import gen_b1024, gen_traj
    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "bench_b1024.npz"))
    Bq, k = gen_b1024.B, gen_b1024.K
    torch.manual_seed(gen_b1024.SEED_MODEL)
    m = tta.EnhancedTwoTowerModel(E, HID)
    with torch.no_grad():
        for prm in m.parameters():
            prm.copy_(_bf16(prm))
    m = m.to(DEV).set_compute_dtype(torch.bfloat16).train()
    q, d = gen_traj.make_batches(Bq, seed=gen_b1024.SEED_DATA, n=1)[0]
    q, d = q.to(DEV), d.to(DEV)
    lib = _lib.load()
    assert lib.tt_gru_fwd_ws_size(_lib.DT_BF16, 4, Bq, T, 2 * HID, 6 * 2 * HID, 2 * 2 * HID) > 0, \
        "the column-split forward must be the auto choice at B 1024"
    for name in ("gru_fwd_xc", "gru_fwd_xs", "gemm_bres", "gemm_persist", "gru_bwd_persist", "hn_gemm"):
        assert _lib.get_option(name) == {"hn_gemm": 0}.get(name, 1), name  # defaults, nothing forced
    crit = tta.HardNegativeMarginLoss(k=k, margin=0.2, compute_dtype=torch.bfloat16)
    torch.manual_seed(gen_b1024.SEED_DROP)
    qv, dv = m(q, d)
    loss = crit(qv, dv)
    tta.check_gru_status()
    idx = crit.last_indices.long().cpu().numpy()
    ridx = gold["picks"].astype(np.int64)
    same = np.array([set(idx[i]) == set(ridx[i]) for i in range(Bq)])
    kth = gold["top16_cos"][:, k - 1]
    worst = 0.0
    for i in np.nonzero(~same)[0]:
        top = dict(zip(gold["top16_idx"][i].astype(np.int64).tolist(), gold["top16_cos"][i].tolist()))
        for j in set(idx[i].tolist()) - set(ridx[i].tolist()):
            assert j in top, (i, j, "GPU pick outside the oracle's 16 best")
            worst = max(worst, float(kth[i] - top[j]))
    lv, rv = float(loss.detach()), float(gold["loss"])
    print(f"B 1024: {same.mean():.4f} of rows mine the oracle's set (worst near-tie gap {worst:.2e}); "
          f"loss {lv:.6f} vs {rv:.6f}")
    assert same.mean() >= 0.90, same.mean()
    assert worst <= 1e-2, worst
    assert rv > 0.01 and abs(lv - rv) <= 5e-3 * abs(rv), (lv, rv)
    rows = torch.from_numpy(gold["rows"])
    for a, b, amax in ((qv, gold["qv"], gold["qv_absmax"]), (dv, gold["dv"], gold["dv_absmax"])):
        err = float((a.detach().cpu()[rows].double() - torch.from_numpy(b).double()).abs().max())
        assert err <= 3e-2 * float(amax), err
    # gradients with the oracle's negatives (explicit-negative branch, same tower kernels)
    del loss
    torch.manual_seed(gen_b1024.SEED_DROP)
    qv, dv = m(q, d)
    from two_towers_amd.losses import _MarginFn  # HardNegativeMarginLoss's margin step, given indices
    oidx = torch.from_numpy(ridx).to(DEV, torch.int32).contiguous()
    loss2 = _MarginFn.apply(qv, dv, oidx, 0, 0.2, 1e-8) / Bq
    m.zero_grad(set_to_none=True)
    loss2.backward()
    tta.check_gru_status()
    assert abs(float(loss2.detach()) - rv) <= 5e-3 * abs(rv), (float(loss2), rv)
    worst_g = (0.0, 1.0, "")
    for name, prm in m.named_parameters():
        pos = torch.from_numpy(gold[f"pos/{name}"])
        a = prm.grad.detach().reshape(-1).cpu()[pos].double()
        b = torch.from_numpy(gold[f"g/{name}"]).double()
        cos = float((a * b).sum() / (a.norm() * b.norm() + 1e-300))
        frob = float((a - b).norm() / (b.norm() + 1e-300))
        cmin, rmax = (0.998, 0.06) if prm.dim() == 2 else (0.996, 0.09)
        assert cos >= cmin and frob <= rmax, (name, cos, frob)
        worst_g = max(worst_g, (frob, cos, name))
    print(f"B 1024 gradients (oracle negatives): worst {worst_g[2]}: rel {worst_g[0]:.4f}, cos {worst_g[1]:.5f}")


def test_bench_composition_bf16_adam_trajectory_matches_oracle():
    """Ten training steps of the bench composition (train_enhanced.py:58-63 with the
    configs[2] loss): EnhancedTwoTowerModel(300, 256), T 64, B 512, bf16 compute, dropout
    0.1, HardNegativeMarginLoss (k 5, margin 0.2), two_towers_amd.Adam (lr gen_traj.LR =
    1e-4, see there), two batches of correlated (query, positive) pairs alternating --
    against the oracle's trajectory (tests/golden/bench_traj.npz, oracle/gen_traj.py:
    cpu_ref forward + mining + margin loss, torch.optim.Adam on fp32 master weights whose
    forward sees their bf16 rounding, the same inputs and the same per-step dropout seeds;
    ~1 minute of CPU per step, so computed once in the build container). The oracle mines
    on its own fp32 outputs: a near-tie picked differently moves a row's mean negative
    cosine by at most ~2e-2 / k, i.e. the loss by ~1e-5.
    Tolerances: per-step loss within 1e-2 relative (5e-3 at step 0, as the single-step
    composition test); at EVERY step, every pick outside the oracle's set is a near-tie of
    the oracle's ranking at that step (its oracle cosine within 2e-2 of the oracle's k-th best;
    the fixture holds each row's 16 best per step) and >= 90 % of the rows pick the oracle's
    exact set at steps 0-1, >= 70 % after (the two trajectories' weights drift apart by a
    fraction of their movement while a row's 5th and 6th best cosines are ~1e-3 apart at B 512:
    measured 0.95, 0.92, then 0.71-0.81); among the rows whose oracle k-th / (k+1)-th gap
    exceeds 2e-3 (27-54 % of them) >= 90 % pick the oracle's set at EVERY step (measured
    0.928-1.0), and every row whose gap exceeds 5e-3 does (measured 1.0 at every step);
    round 5's fixture, lr 1e-3 on uncorrelated pairs,
    drove the loss onto the 0.2 margin floor where every document is a near-tie: 0.96 at step
    0, 0.01 by step 9); the oracle's loss ends below the 0.2 margin (the towers separate
    positives from negatives, no collapse); for every
    tensor, at 64 fixed positions, the distance of the final weights from the oracle's at
    most 0.25 of the distance the oracle's ten steps moved them (Adam's early steps are
    ~lr * sign(g): an element whose gradient is near zero can move the other way)."""
    import os
    from oracle import gen_traj
    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "bench_traj.npz"))
    Bq, k, steps, lr = gen_traj.B, gen_traj.K, gen_traj.STEPS, gen_traj.LR
    m, _ = _model(gen_traj.SEED_MODEL)
    m.train()
    batches = gen_traj.make_batches(Bq)
    w0 = {kk: v.detach().cpu().reshape(-1).clone() for kk, v in m.state_dict().items()}
    for kk, v in w0.items():  # same initial weights as the oracle's run
        assert np.array_equal(v[gold[f"pos/{kk}"]].numpy(), gold[f"w0/{kk}"]), kk
    crit = tta.HardNegativeMarginLoss(k=k, margin=0.2, compute_dtype=torch.bfloat16)
    opt = tta.Adam(m.parameters(), lr=lr)
    torch.manual_seed(gen_traj.SEED_DROP)  # the model draws each step's dropout seeds from this stream, as the oracle did
    gl, agree, tiegap, decided = [], [], [], []
    for s in range(steps):
        q, d = batches[s % 2]
        opt.zero_grad()
        loss = crit(*m(q.to(DEV), d.to(DEV)))
        loss.backward()
        opt.step()
        gl.append(float(loss.detach()))
        idx = crit.last_indices.long().cpu().numpy()
        ridx = gold["picks"][s].astype(np.int64)
        same = np.array([set(idx[i]) == set(ridx[i]) for i in range(Bq)])
        agree.append(float(same.mean()))
        # agreement on the rows whose oracle k-th / (k+1)-th gap exceeds 2e-3 and 5e-3 (sets
        # the oracle decides by more than the two trajectories' drift)
        row = []
        for thr in (2e-3, 5e-3):
            dec = gold["gaps"][s] > thr
            row += [float(same[dec].mean()) if dec.any() else 1.0, float(dec.mean())]
        decided.append(row)
        # every pick outside the oracle's set is a near-tie of the oracle's ranking at this step
        kth = gold["top16_cos"][s][:, k - 1]
        worst = 0.0
        for i in np.nonzero(~same)[0]:
            top = dict(zip(gold["top16_idx"][s][i].astype(np.int64).tolist(), gold["top16_cos"][s][i].tolist()))
            for j in set(idx[i].tolist()) - set(ridx[i].tolist()):
                worst = max(worst, float(kth[i] - top[j]) if j in top else float("inf"))
        tiegap.append(worst)
    tta.check_gru_status()
    rl = gold["losses"]
    for s in range(steps):
        print(f"step {s}: loss {gl[s]:.6f} vs oracle {rl[s]:.6f} (rel {abs(gl[s] - rl[s]) / abs(rl[s]):.2e}), "
              f"picks agree {agree[s]:.4f} (rows with gap > 2e-3: {decided[s][0]:.4f} of {decided[s][1]:.3f}; "
              f"> 5e-3: {decided[s][2]:.4f} of {decided[s][3]:.3f}), "
              f"worst near-tie gap {tiegap[s]:.2e}")
    assert float(rl.min()) > 0.01, "hinges inactive: the test would compare zeros"
    # the oracle's towers learn to rank each positive above its mined negatives (loss under the
    # 0.2 margin) instead of collapsing onto the margin floor, where every pick is a near-tie
    assert float(rl[-1]) < 0.2, float(rl[-1])
    for s in range(steps):
        assert tiegap[s] <= 2e-2, (s, tiegap[s])  # a differing pick is always a near-tie ...
        assert agree[s] >= (0.90 if s < 2 else 0.70), (s, agree[s])  # ... and most rows pick the same set
        assert decided[s][0] >= 0.90, (s, decided[s])  # rows the oracle decides by > 2e-3 ...
        assert decided[s][2] == 1.0, (s, decided[s])  # ... and by > 5e-3: all of them
        tol = 5e-3 if s == 0 else 1e-2
        assert abs(gl[s] - rl[s]) <= tol * abs(rl[s]), (s, gl[s], rl[s])
    worst, wk = 0.0, ""
    for kk, v in m.state_dict().items():
        pos = gold[f"pos/{kk}"]
        a = v.detach().cpu().reshape(-1)[pos].double().numpy()
        b, a0 = gold[f"w1/{kk}"].astype(np.float64), gold[f"w0/{kk}"].astype(np.float64)
        r = float(np.linalg.norm(a - b) / (np.linalg.norm(b - a0) + 1e-30))
        if r > worst:
            worst, wk = r, kk
    print(f"final weights: worst ||w - w_ref|| / ||w_ref - w0|| = {worst:.3e} ({wk})")
    assert worst <= 0.25, (wk, worst)
