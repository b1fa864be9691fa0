"""tt_infonce_bwd (the backward of InfoNCELoss / the in-batch MarginRankingLoss branch,
enhanced_two_tower.py:67-82, :84-101) through the C ABI. bf16 with h in {128, 256} runs
the fused backward that recomputes the score tiles and never writes dS
(infonce_bwd_flash_kernel, both roles, split sweeps summed from fp32 slabs); option
infonce_flash = 0 runs the materialised-dS path. Both are checked against a float64
reference of the same rule on the bf16-rounded operands:
    S = inv_tau q d^T - offdiag [j != label_i],  dS = g (softmax(S) - onehot(label)),
    dq = inv_tau dS d,  dd = inv_tau dS^T q.
Tolerance: dS is rounded to bf16 before the second product in both paths (the MFMA
operand), so max-abs error <= 1.5e-2 of the largest gradient entry, cosine >= 0.9999."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from two_towers_amd import _lib  # noqa: E402
from two_towers_amd._lib import call, dtype_code, option  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def ref_grads(q, d, inv_tau, offdiag, lab0, g):
    q64, d64 = q.double(), d.double()
    s = inv_tau * (q64 @ d64.t())
    rows = torch.arange(q.shape[0])
    mask = torch.ones_like(s)
    mask[rows, lab0 + rows] = 0.0
    s = s - offdiag * mask
    p = torch.softmax(s, dim=1)
    p[rows, lab0 + rows] -= 1.0
    ds = g * p
    return inv_tau * ds @ d64, inv_tau * ds.t() @ q64


def run_bwd(q, d, inv_tau, offdiag, lab0, g, flash):
    lib = _lib.load()
    B, h = q.shape
    nd = d.shape[0]
    qd, dd = q.to(DEV, BF).contiguous(), d.to(DEV, BF).contiguous()
    st = torch.cuda.current_stream().cuda_stream
    lse = torch.empty(B, device=DEV)
    row = torch.empty(B, device=DEV)
    wsf = torch.empty(lib.tt_infonce_fwd_ws_size(B, nd), dtype=torch.uint8, device=DEV)
    call("tt_infonce_fwd", dtype_code(BF), qd.data_ptr(), B, dd.data_ptr(), nd, h, inv_tau, offdiag, lab0,
         lse.data_ptr(), row.data_ptr(), wsf.data_ptr(), st)
    gdev = torch.tensor([g], device=DEV)
    dq = torch.full((B, h), float("nan"), device=DEV)
    ddn = torch.full((nd, h), float("nan"), device=DEV)
    with option("infonce_flash", flash):
        ws = torch.empty(lib.tt_infonce_bwd_ws_size(dtype_code(BF), B, nd, h), dtype=torch.uint8, device=DEV)
        call("tt_infonce_bwd", dtype_code(BF), qd.data_ptr(), B, dd.data_ptr(), nd, h, inv_tau, offdiag, lab0,
             lse.data_ptr(), gdev.data_ptr(), dq.data_ptr(), ddn.data_ptr(), ws.data_ptr(), st)
        torch.cuda.synchronize()
    return dq.cpu(), ddn.cpu(), qd.float().cpu(), dd.float().cpu()


CASES = [  # B, nd, h, label offset, offdiag
    (256, 256, 256, 0, 0.0),      # InfoNCE, one tile per split
    (300, 1000, 128, 0, 0.0),     # tails on both operands
    (130, 4100, 256, 2048, 0.1),  # DP rank 1 of 2 with the margin branch's off-diagonal shift
    (64, 8192, 256, 0, 0.0),      # one own block, the sweep split over 128 workgroups
    (2048, 2048, 128, 0, 0.0),    # 16 own blocks x 16 splits
]


@pytest.mark.parametrize("flash", [1, 0])
@pytest.mark.parametrize("B,nd,h,lab0,offdiag", CASES)
def test_infonce_bwd_matches_float64(B, nd, h, lab0, offdiag, flash):
    gen = torch.Generator().manual_seed(B + 7 * nd + h)
    q = torch.nn.functional.normalize(torch.randn(B, h, generator=gen), dim=1)
    d = torch.nn.functional.normalize(torch.randn(nd, h, generator=gen), dim=1)
    inv_tau, g = 1 / 0.07, 1.0 / B
    dq, dd, qr, dr = run_bwd(q, d, inv_tau, offdiag, lab0, g, flash)
    rq, rd = ref_grads(qr, dr, inv_tau, offdiag, lab0, g)
    for got, ref in ((dq, rq), (dd, rd)):
        assert torch.isfinite(got).all()
        err = float((got.double() - ref).abs().max() / ref.abs().max())
        cos = float((got.double() * ref).sum() / (got.double().norm() * ref.norm()))
        assert err <= 1.5e-2 and cos >= 0.9999, (err, cos)


def test_flash_and_materialised_paths_agree():
    """The fused and the materialised-dS backward round dS the same way, so at B = N =
    1024 they agree far inside the float64 tolerance."""
    gen = torch.Generator().manual_seed(5)
    q = torch.nn.functional.normalize(torch.randn(1024, 256, generator=gen), dim=1)
    d = torch.nn.functional.normalize(torch.randn(1024, 256, generator=gen), dim=1)
    a = run_bwd(q, d, 1 / 0.07, 0.0, 0, 1 / 1024, 1)
    b = run_bwd(q, d, 1 / 0.07, 0.0, 0, 1 / 1024, 0)
    for x, y in zip(a[:2], b[:2]):
        assert float((x - y).abs().max() / y.abs().max()) < 2e-3


def test_infonce_configs3_rank_shape_matches_float64():
    """configs[3] per-rank shape: 8192 local queries scored against the 65,536-row global
    pool (rank 3 of 8, labels at 3 * 8192 + i), InfoNCE (tau 0.07). Forward: the per-row
    LSE and loss against float64 (relative 1e-5 / absolute 2e-4 of the bf16-operand
    scores); backward (fused, no dS): the tolerances stated at the top of this file. The
    float64 reference runs on the GPU."""
    B, nd, h, lab0 = 8192, 65536, 256, 3 * 8192
    gen = torch.Generator().manual_seed(83)
    q = torch.nn.functional.normalize(torch.randn(B, h, generator=gen), dim=1)
    d = torch.nn.functional.normalize(torch.randn(nd, h, generator=gen), dim=1)
    inv_tau, g = 1 / 0.07, 1.0 / B
    lib = _lib.load()
    qd, dd = q.to(DEV, BF).contiguous(), d.to(DEV, BF).contiguous()
    st = torch.cuda.current_stream().cuda_stream
    lse = torch.empty(B, device=DEV)
    row = torch.empty(B, device=DEV)
    wsf = torch.empty(lib.tt_infonce_fwd_ws_size(B, nd), dtype=torch.uint8, device=DEV)
    call("tt_infonce_fwd", dtype_code(BF), qd.data_ptr(), B, dd.data_ptr(), nd, h, inv_tau, 0.0, lab0,
         lse.data_ptr(), row.data_ptr(), wsf.data_ptr(), st)
    gdev = torch.tensor([g], device=DEV)
    dq = torch.full((B, h), float("nan"), device=DEV)
    ddn = torch.full((nd, h), float("nan"), device=DEV)
    ws = torch.empty(lib.tt_infonce_bwd_ws_size(dtype_code(BF), B, nd, h), dtype=torch.uint8, device=DEV)
    call("tt_infonce_bwd", dtype_code(BF), qd.data_ptr(), B, dd.data_ptr(), nd, h, inv_tau, 0.0, lab0,
         lse.data_ptr(), gdev.data_ptr(), dq.data_ptr(), ddn.data_ptr(), ws.data_ptr(), st)
    torch.cuda.synchronize()
    q64, d64 = qd.double(), dd.double()
    s = inv_tau * (q64 @ d64.t())
    rows = torch.arange(B, device=DEV)
    rlse = torch.logsumexp(s, dim=1)
    rrow = rlse - s[rows, lab0 + rows]
    assert float((lse.double() - rlse).abs().max()) <= 1e-5 * float(rlse.abs().max()) + 2e-4
    assert float((row.double() - rrow).abs().max()) <= 2e-4
    p = torch.softmax(s, dim=1)
    del s
    p[rows, lab0 + rows] -= 1.0
    p *= g
    rq = inv_tau * (p @ d64)
    rd = inv_tau * (p.t() @ q64)
    del p
    for got, ref in ((dq, rq), (ddn, rd)):
        assert torch.isfinite(got).all()
        err = float((got.double() - ref).abs().max() / ref.abs().max())
        cos = float((got.double() * ref).sum() / (got.double().norm() * ref.norm()))
        assert err <= 1.5e-2 and cos >= 0.9999, (err, cos)
