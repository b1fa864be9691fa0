"""The NS-stage product ring of the 2-stage LDS-DMA loop (tt_gemm_core.h DLoop NS) only
changes when each K-tile's DMAs are waited for, never the MFMA order: the per-step GRU
kernels (option gru_step_ring) must be bit-identical to their double-buffered form at
grids of at most one workgroup per CU (where the ring is used)."""
import pytest
import torch

from two_towers_amd._lib import GruBwdRec, GruFwdRec, call, load, option, stream_ptr

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _gru_once(dt, B, T, H, ring, bwd_rows=0):
    """One per-step forward + backward over 4 recurrences (fp32: the per-step kernels)."""
    code = 0 if dt == torch.float32 else 1
    g = torch.Generator(device=DEV).manual_seed(71)
    G = torch.randn(B * T, 6 * H, device=DEV, generator=g).to(dt)
    whh = [(torch.randn(3 * H, H, device=DEV, generator=g) * H ** -0.5).to(dt) for _ in range(4)]
    bhn = [torch.randn(H, device=DEV, generator=g) * 0.1 for _ in range(4)]
    Y = [torch.empty(B * T, 2 * H, device=DEV, dtype=dt) for _ in range(2)]
    S = [torch.empty(B * T, 4 * H, device=DEV, dtype=dt) for _ in range(4)]
    hs = [torch.empty(2, B, H, device=DEV) for _ in range(4)]
    recs = (GruFwdRec * 4)()
    for i in range(4):
        ti, d = divmod(i, 2)
        r = recs[i]
        r.g = G[:, d * 3 * H:].data_ptr()
        r.whh = whh[i].data_ptr()
        r.bhn = bhn[i].data_ptr()
        r.y = Y[ti][:, d * H:].data_ptr()
        r.x1 = None
        r.save = S[i].data_ptr()
        r.hstate = hs[i].data_ptr()
        r.dir = d
    st = stream_ptr(torch.device(DEV))
    dY = [torch.randn(B * T, 2 * H, device=DEV, generator=g).to(dt) * 0.01 for _ in range(2)]
    dG = [torch.empty(B * T, 8 * H, device=DEV, dtype=dt) for _ in range(2)]
    dhs = [torch.empty(2, B, H, device=DEV, dtype=dt) for _ in range(4)]
    nbr = load().tt_gru_bias_rows(B)
    part = [torch.empty(nbr, 4 * H, device=DEV) for _ in range(4)]
    brecs = (GruBwdRec * 4)()
    for i in range(4):
        ti, d = divmod(i, 2)
        r = brecs[i]
        r.save = S[i].data_ptr()
        r.y = Y[ti][:, d * H:].data_ptr()
        r.dy = dY[ti][:, d * H:].data_ptr()
        r.dfinal = None
        r.whh = whh[i].data_ptr()
        r.dgx = dG[ti][:, d * 3 * H:].data_ptr()
        r.dgh = dG[ti][:, 6 * H + d * H:].data_ptr()
        r.dhstate = dhs[i].data_ptr()
        r.dbias_part = part[i].data_ptr()
        r.dir = d
    with option("gru_step_ring", ring), option("gru_step", 1), option("gru_bwd_persist", 0), \
            option("gru_bwd_rows", bwd_rows):
        call("tt_gru_fwd", code, recs, 4, B, T, H, 6 * H, 2 * H, 0.0, None, 0, st)
        call("tt_gru_bwd", code, brecs, 4, B, T, H, 2 * H, 8 * H, 0, st)
    torch.cuda.synchronize()
    return [y.clone() for y in Y] + [s.clone() for s in S] + [d.clone() for d in dG] + [p.clone() for p in part]


@pytest.mark.parametrize("bwd_rows", [0, 128])  # 0: the host's pick (64-row tiles here)
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gru_step_ring_is_bit_identical(dt, bwd_rows):
    B, T, H = 256, 8, 256  # forward 4 x 2 x 4 = 32 workgroups, backward 2 x 4 x 2 x 2: one per CU
    a = _gru_once(dt, B, T, H, 2, bwd_rows)
    b = _gru_once(dt, B, T, H, 4, bwd_rows)
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x, y), i
