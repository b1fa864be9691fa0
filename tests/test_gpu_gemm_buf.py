"""The 256x256 GEMM's operand DMAs through buffer resources (option gemm_buf, Loop8 BUF)
against the per-lane-pointer DMAs (gemm_buf 0): the LDS images of every consumed K-tile
are the same bytes, so C must be bit-identical, on each path that runs the 8-phase loop --
the persistent short-K kernel (input projections), the long-K kernel (dX), split-K TN
with the split-column A and the time-shifted B (dW_hh) -- with ragged M and N; and equal
to a fp32 product of the bf16-rounded operands."""
import pytest
import torch

from two_towers_amd import ops
from two_towers_amd._lib import option

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _both(fn):
    outs = []
    for buf in (0, 1):
        with option("gemm_buf", buf):
            outs.append(fn())
    torch.cuda.synchronize()
    return outs


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-12))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("akout,bkout", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("path", ["persist", "long_k"])
def test_buffer_dma_gemm_is_bit_identical(akout, bkout, path, dt):
    # persist: >= 512 tiles of 256^2 at <= 24 K-tiles; long_k: past the persistent cap
    if dt == torch.bfloat16:
        m, n, k = (8200, 4136, 1024) if path == "persist" else (4200, 4136, 2048)
    else:  # fp32 K-tiles are 32 deep
        m, n, k = (8200, 4136, 512) if path == "persist" else (4200, 4136, 1024)
    g = torch.Generator().manual_seed(31 + 2 * akout + bkout)
    A = torch.randn(m, k, generator=g).to(dt)
    B = torch.randn(n, k, generator=g).to(dt)
    bias = torch.randn(n, generator=g).to(DEV)
    Ad = (A.t().contiguous() if akout else A).to(DEV)
    Bd = (B.t().contiguous() if bkout else B).to(DEV)

    def run():
        C = torch.empty(m, n, device=DEV, dtype=dt)
        ops.gemm([Ad], [Bd], [C], m=m, n=n, k=k, lda=m if akout else k, ldb=n if bkout else k, ldc=n,
                 a_kouter=bool(akout), b_kouter=bool(bkout), dtype=dt, out_dtype=dt, bias=[bias], splits=1)
        return C

    c0, c1 = _both(run)
    assert torch.equal(c0, c1)
    ref = A.to(DEV).double() @ B.to(DEV).double().t() + bias.double()
    assert _rel(c1.double(), ref) < (1e-2 if dt == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("T", [32, 64, 128])
def test_buffer_dma_split_k_wgrad_hh_composition(T):
    """dW_hh's GEMM: A = dL/dgh^T through the split-column loader (r|z columns of dG, the
    W_hn block at column 6H), B = h_{t-1} (time-shifted: the masked k-rows are the same lanes
    of every K-tile at T 32 / 64, one k-row of every other K-tile at T 128), split-K."""
    H, K = 256, 16384
    Bsz = K // T
    g = torch.Generator().manual_seed(41 + T)
    dG = torch.randn(K, 8 * H, generator=g).to(torch.bfloat16).to(DEV)
    Y = torch.randn(K, 2 * H, generator=g).to(torch.bfloat16).to(DEV)
    a = [dG[:, d * 3 * H:] for d in range(2)]
    a_hi = [dG[:, 6 * H + d * H:] for d in range(2)]
    b = [Y[:, d * H:] for d in range(2)]

    def run():
        C = [torch.empty(3 * H, H, device=DEV) for _ in range(2)]
        ops.gemm(a, b, C, m=3 * H, n=H, k=K, lda=8 * H, ldb=2 * H, ldc=H, a_kouter=True, b_kouter=True,
                 dtype=torch.bfloat16, out_dtype=torch.float32, bshift=[-1, 1], seq_t=T, a_hi=a_hi, a_split=2 * H)
        return C

    c0, c1 = _both(run)
    for d in range(2):
        assert torch.equal(c0[d], c1[d]), d
        dgh = torch.cat([a[d][:, :2 * H], a_hi[d][:, :H]], 1).float()
        h = b[d][:, :H].float().reshape(Bsz, T, H)
        hs = torch.zeros_like(h)
        if d == 0:
            hs[:, 1:] = h[:, :-1]
        else:
            hs[:, :-1] = h[:, 1:]
        ref = dgh.t() @ hs.reshape(K, H)
        assert _rel(c1[d], ref) < 1e-5, (d, _rel(c1[d], ref))


def test_persistent_tile_order_is_bit_identical():
    """gemm_persist's column-group-per-XCD tile walk (option gemm_order 1) computes every
    tile exactly as the row-panel walk (0) does: the input-projection shape class, two batch
    entries, 12 column panels (3 groups of 4), 64 row panels."""
    m, n, k = 16384, 3072, 1024
    g = torch.Generator().manual_seed(51)
    A = [torch.randn(m, k, generator=g).to(torch.bfloat16).to(DEV) for _ in range(2)]
    B = [torch.randn(n, k, generator=g).to(torch.bfloat16).to(DEV) for _ in range(2)]
    bias = [torch.randn(n, generator=g).to(DEV) for _ in range(2)]
    outs = []
    for order in (0, 1):
        C = [torch.empty(m, n, device=DEV, dtype=torch.bfloat16) for _ in range(2)]
        with option("gemm_order", order):
            ops.gemm(A, B, C, m=m, n=n, k=k, lda=k, ldb=k, ldc=n, a_kouter=False, b_kouter=False,
                     dtype=torch.bfloat16, out_dtype=torch.bfloat16, bias=bias, splits=1)
        outs.append(C)
    torch.cuda.synchronize()
    for i in range(2):
        assert torch.equal(outs[0][i], outs[1][i]), i
        ref = A[i].float() @ B[i].float().t() + bias[i]
        assert _rel(outs[1][i].float(), ref) < 1e-2
