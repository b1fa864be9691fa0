"""Kernel-level parity on the GPU: tt_gemm layouts, GRU layer, head, losses, Adam.

Reference for every floating-point kernel is plain PyTorch fp32 / fp64 on the CPU
(the oracle's arithmetic). Tolerances: fp32 kernels rtol 1e-4-ish (accumulation
order differs), bf16 kernels ~2e-2 relative to the output scale.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from two_towers_amd import ops  # noqa: E402

DEV = "cuda"


def rel_err(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("akout,bkout", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("m,n,k", [(128, 128, 64), (200, 136, 72), (384, 256, 640), (64, 40, 1000)])
def test_gemm_layouts(dt, akout, bkout, m, n, k):
    g = torch.Generator().manual_seed(m * 7 + n * 3 + k)
    A = torch.randn(m, k, generator=g)
    B = torch.randn(n, k, generator=g)
    ref = A @ B.t()
    Ad = (A.t().contiguous() if akout else A).to(DEV, dt)
    Bd = (B.t().contiguous() if bkout else B).to(DEV, dt)
    C = torch.empty(m, n, device=DEV)
    ops.gemm([Ad], [Bd], [C], m=m, n=n, k=k, lda=m if akout else k, ldb=n if bkout else k, ldc=n,
             a_kouter=bool(akout), b_kouter=bool(bkout), dtype=dt, out_dtype=torch.float32, splits=1)
    refq = (A.to(dt).float() @ B.to(dt).float().t())
    tol = 1e-5 if dt == torch.float32 else 1e-3
    assert rel_err(C, refq) < tol, rel_err(C, refq)
    assert rel_err(C, ref) < (1e-5 if dt == torch.float32 else 2e-2)


@pytest.mark.parametrize("a3", [0, 1])
@pytest.mark.parametrize("akout,bkout,dt", [(0, 0, torch.bfloat16), (0, 1, torch.bfloat16), (1, 0, torch.bfloat16),
                                            (1, 1, torch.bfloat16), (0, 0, torch.float32)])
def test_gemm_big_tiles(akout, bkout, dt, a3):
    """>= 256 tiles of 256x256 with a long K run the 8-phase loop of gemm_kernel (not the
    persistent short-K kernel): ragged M/N/K tails, bias, alpha; a3 1: A prefetched two
    K-tiles ahead through a 3-slot ring (option gemm_a3), 0: the 2-slot schedule."""
    from two_towers_amd._lib import option
    m, n, k = 4200, 4136, 2056
    g = torch.Generator().manual_seed(21)
    A = torch.randn(m, k, generator=g).to(dt).float()
    B = torch.randn(n, k, generator=g).to(dt).float()
    bias = torch.randn(n, generator=g)
    Ad = (A.t().contiguous() if akout else A).to(DEV, dt)
    Bd = (B.t().contiguous() if bkout else B).to(DEV, dt)
    C = torch.empty(m, n, device=DEV)
    with option("gemm_a3", a3):
        ops.gemm([Ad], [Bd], [C], m=m, n=n, k=k, lda=m if akout else k, ldb=n if bkout else k, ldc=n,
                 a_kouter=bool(akout), b_kouter=bool(bkout), dtype=dt, out_dtype=torch.float32, bias=[bias.to(DEV)],
                 alpha=0.5, splits=1)
    ref = 0.5 * (A @ B.t()) + bias
    assert rel_err(C, ref) < 1e-5, rel_err(C, ref)


@pytest.mark.parametrize("a3", [0, 1])
def test_gemm_big_tiles_splitk_tn(a3):
    """The weight-gradient shape class: TN (both operands K-outer), split-K over >= 256
    workgroups of 256x256 tiles, fp32 partials summed by splitk_reduce_kernel."""
    from two_towers_amd._lib import option
    m, n, k = 1536, 1032, 16384
    g = torch.Generator().manual_seed(22)
    A = torch.randn(k, m, generator=g).to(torch.bfloat16).float()
    B = torch.randn(k, n, generator=g).to(torch.bfloat16).float()
    C = torch.empty(m, n, device=DEV)
    with option("gemm_a3", a3):
        ops.gemm([A.to(DEV, torch.bfloat16)], [B.to(DEV, torch.bfloat16)], [C], m=m, n=n, k=k, lda=m, ldb=n, ldc=n,
                 a_kouter=True, b_kouter=True, dtype=torch.bfloat16, out_dtype=torch.float32)  # splits picked: 17
    ref = A.t() @ B
    assert rel_err(C, ref) < 1e-5, rel_err(C, ref)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_splitk_bias_accum(dt):
    g = torch.Generator().manual_seed(1)
    m, n, k = 256, 192, 4096
    A = torch.randn(k, m, generator=g)  # K-outer
    B = torch.randn(k, n, generator=g)
    bias = torch.randn(n, generator=g)
    C0 = torch.randn(m, n, generator=g)
    C = C0.clone().to(DEV)
    ops.gemm([A.to(DEV, dt)], [B.to(DEV, dt)], [C], m=m, n=n, k=k, lda=m, ldb=n, ldc=n, a_kouter=True,
             b_kouter=True, dtype=dt, out_dtype=torch.float32, bias=[bias.to(DEV)], alpha=0.5, accumulate=True,
             splits=8)
    ref = 0.5 * (A.to(dt).float().t() @ B.to(dt).float()) + bias + C0
    assert rel_err(C, ref) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_batched_shift(dt):
    """B operand row k -> k+shift within blocks of T (GRU h_{t-1} operand)."""
    g = torch.Generator().manual_seed(2)
    Bsz, T, M, N = 16, 8, 48, 32
    K = Bsz * T
    A = [torch.randn(K, M, generator=g) for _ in range(2)]
    Bm = [torch.randn(K, N, generator=g) for _ in range(2)]
    C = [torch.empty(M, N, device=DEV) for _ in range(2)]
    ops.gemm([a.to(DEV, dt) for a in A], [b.to(DEV, dt) for b in Bm], C, m=M, n=N, k=K, lda=M, ldb=N, ldc=N,
             a_kouter=True, b_kouter=True, dtype=dt, out_dtype=torch.float32, bshift=[-1, 1], seq_t=T, splits=1)
    for i, sh in enumerate((-1, 1)):
        Bs = Bm[i].to(dt).float().view(Bsz, T, N)
        shifted = torch.zeros_like(Bs)
        if sh == -1:
            shifted[:, 1:] = Bs[:, :-1]
        else:
            shifted[:, :-1] = Bs[:, 1:]
        ref = A[i].to(dt).float().t() @ shifted.view(K, N)
        assert rel_err(C[i], ref) < 1e-5, (i, rel_err(C[i], ref))


def test_gemm_dropout_epilogue():
    from oracle.cpu_ref import dropout_mask
    g = torch.Generator().manual_seed(3)
    m, n, k = 130, 64, 32
    A = torch.randn(m, k, generator=g)
    B = torch.randn(n, k, generator=g)
    C = torch.empty(m, n, device=DEV)
    ops.gemm([A.to(DEV)], [B.to(DEV)], [C], m=m, n=n, k=k, lda=k, ldb=k, ldc=n, a_kouter=False, b_kouter=False,
             dtype=torch.float32, out_dtype=torch.float32, drop_seed=1234, drop_p=0.1)
    mask = torch.from_numpy(dropout_mask(1234, m, n, 0.1))
    ref = (A @ B.t()) * mask
    assert rel_err(C, ref) < 1e-5
    frac = float((mask == 0).float().mean())
    assert 0.05 < frac < 0.15


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_embed_gather(dt):
    V, E = 1000, 300
    ep = ops.pad_cols(E, dt)
    table = torch.zeros(V, ep, dtype=dt)
    table[:, :E] = torch.randn(V, E).to(dt)
    ids = torch.randint(-1, V, (517,), dtype=torch.int32)
    out = torch.empty(517, ep, dtype=dt, device=DEV)
    ops.embed_gather(table.to(DEV), ids.to(DEV), out)
    ref = torch.where((ids >= 0)[:, None], table[ids.clamp_min(0).long()], torch.zeros(1, ep, dtype=dt))
    assert torch.equal(out.cpu(), ref)


def test_adam_matches_torch():
    from two_towers_amd.optim import Adam
    torch.manual_seed(0)
    ps = [torch.randn(s) for s in [(7, 5), (300,), (4097,), (3, 3, 3)]]
    gs = [[torch.randn_like(p) for p in ps] for _ in range(3)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    mine = [torch.nn.Parameter(p.clone().to(DEV)) for p in ps]
    o1 = torch.optim.Adam(ref, lr=1e-2)
    o2 = Adam(mine, lr=1e-2)
    for step in range(3):
        for p, g in zip(ref, gs[step]):
            p.grad = g.clone()
        for p, g in zip(mine, gs[step]):
            p.grad = g.clone().to(DEV)
        o1.step()
        o2.step()
    for a, b in zip(ref, mine):
        assert torch.allclose(a.detach(), b.detach().cpu(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("akout,bkout", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("out", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n", [4104, 4100])
def test_gemm_persistent_tiles(akout, bkout, out, n):
    """Shapes with >= 512 256x256 tiles and a short K run the persistent kernel (K-tile
    stream across tiles): ragged M/N/K tails, bias, relu, two batch entries; compared
    with fp32 math on the same bf16-rounded operands; n = 4100 leaves rows that are not
    16-byte aligned (element stores)."""
    if bkout and n % 8:
        pytest.skip("a K-outer B needs 16-byte rows (ldb = n)")
    dt = torch.bfloat16
    m, k = 8200, 136
    g = torch.Generator().manual_seed(5)
    As = [torch.randn(m, k, generator=g).to(dt).float() for _ in range(2)]
    Bs = [torch.randn(n, k, generator=g).to(dt).float() for _ in range(2)]
    bias = [torch.randn(n, generator=g) for _ in range(2)]
    Ad = [(a.t().contiguous() if akout else a).to(DEV, dt) for a in As]
    Bd = [(b.t().contiguous() if bkout else b).to(DEV, dt) for b in Bs]
    C = [torch.empty(m, n, device=DEV, dtype=out) for _ in range(2)]
    ops.gemm(Ad, Bd, C, m=m, n=n, k=k, lda=m if akout else k, ldb=n if bkout else k, ldc=n, a_kouter=bool(akout),
             b_kouter=bool(bkout), dtype=dt, out_dtype=out, bias=[b.to(DEV) for b in bias], relu=True, splits=1)
    for i in range(2):
        ref = torch.relu(As[i] @ Bs[i].t() + bias[i])
        tol = 1e-5 if out == torch.float32 else 8e-3
        assert rel_err(C[i].float(), ref) < tol, (i, rel_err(C[i].float(), ref))


@pytest.mark.parametrize("stream", [0, 1])
def test_gemm_persistent_bf16_output_is_rounded_fp32(stream):
    """The persistent kernel's direct epilogue (transposed accumulators, bf16 pairs
    exchanged between column tiles by v_permlane16_swap): its bf16 output must be exactly
    the bf16 rounding of its own fp32 output, element by element, with bias, alpha and
    dropout applied; stream 1 is large enough (>= 64 MiB of output) for the write-through
    store form. A wrong lane -> column map moves values between columns and fails here
    even where a relative-error check could not see it."""
    from two_towers_amd._lib import option
    dt = torch.bfloat16
    m, n, k = (16640, 4352, 136) if stream else (8448, 4352, 200)  # >= 512 tiles
    g = torch.Generator().manual_seed(11 + stream)
    A = torch.randn(m, k, generator=g).to(DEV, dt)
    B = torch.randn(n, k, generator=g).to(DEV, dt)
    bias = torch.randn(n, generator=g).to(DEV)
    outs = {}
    for out in (torch.float32, torch.bfloat16):
        C = torch.empty(m, n, device=DEV, dtype=out)
        with option("gemm_stream_out", stream):
            ops.gemm([A], [B], [C], m=m, n=n, k=k, lda=k, ldb=k, ldc=n, a_kouter=False, b_kouter=False, dtype=dt,
                     out_dtype=out, bias=[bias], alpha=0.75, drop_seed=77, drop_p=0.1, splits=1)
        outs[out] = C
    want = outs[torch.float32].to(torch.bfloat16)
    bad = int((outs[torch.bfloat16].view(torch.int16) != want.view(torch.int16)).sum())
    assert bad == 0, f"{bad} of {m * n} bf16 outputs differ from the rounded fp32 outputs"
    ref = 0.75 * (A.float() @ B.float().t()) + bias
    got = outs[torch.float32]
    kept = got != 0
    assert rel_err(got[kept] / (1 / 0.9), ref[kept]) < 1e-5
    frac = 1 - float(kept.float().mean())
    assert 0.08 < frac < 0.12, frac


@pytest.mark.parametrize("m,n,k,nb,with_bias", [(524288, 3072, 320, 2, True), (70000, 3072, 320, 2, True),
                                                (65579, 1536, 96, 1, False), (40000, 384, 352, 2, True)])
@pytest.mark.parametrize("rows", [32, 64])
def test_gemm_b_resident_matches_persistent(m, n, k, nb, with_bias, rows):
    """gemm_bres (the layer-0 input projection: each workgroup keeps a 192-column panel of
    B in LDS, its waves walk 32-row A tiles (8 waves) or 64-row tiles (4 waves, option
    bres_rows 64) with no barrier) against the persistent 256x256
    kernel (option gemm_bres = 0) on the same operands: the same MFMA instruction, operand
    roles and k order, so every bf16 output must be identical. The bench shape (M = B*T
    = 524,288, N = 6H = 3072, K = Ep = 320, two towers) and shapes whose rows do not fill
    the 32-row tiles of the 8 row groups, with and without bias, K 96 and 352 (a partial
    64-deep K-tile image)."""
    from two_towers_amd._lib import option
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(m + n + k)
    A = [torch.randn(m, k, generator=g, device=DEV).to(dt) for _ in range(nb)]
    B = [(torch.randn(n, k, generator=g, device=DEV) * k ** -0.5).to(dt) for _ in range(nb)]
    bias = [torch.randn(n, generator=g, device=DEV) for _ in range(nb)] if with_bias else None
    outs = []
    for br in (1, 0):
        C = [torch.full((m, n), float("nan"), device=DEV, dtype=dt) for _ in range(nb)]
        with option("gemm_bres", br), option("bres_rows", rows):
            ops.gemm(A, B, C, m=m, n=n, k=k, lda=k, ldb=k, ldc=n, a_kouter=False, b_kouter=False, dtype=dt,
                     out_dtype=dt, bias=bias, splits=1)
        torch.cuda.synchronize()
        outs.append(C)
    for i in range(nb):
        bad = int((outs[0][i].view(torch.int16) != outs[1][i].view(torch.int16)).sum())
        assert bad == 0, f"batch {i}: {bad} of {m * n} outputs differ"
    # and against fp32 math on a sample of rows
    rows = torch.randint(0, m, (512,), generator=g, device=DEV)
    ref = A[0][rows].float() @ B[0].float().t() + (bias[0] if with_bias else 0)
    assert rel_err(outs[0][0][rows].float(), ref) < 8e-3


@pytest.mark.parametrize("m,n,k,nb,with_bias", [(70144, 3072, 1024, 2, True), (4096, 512, 64, 1, False),
                                                (16384, 1536, 640, 2, True)])
@pytest.mark.parametrize("form", [1, 2])
def test_gemm_four_wave_kernel_matches_persistent(m, n, k, nb, with_bias, form):
    """The four-wave 128x128-per-wave NT kernel (option gemm_w4: 1 LDS-DMA operand staging,
    2 register staging) against the persistent
    256x256 kernel on the same operands: same MFMA instruction, operand order (transposed
    accumulate) and k order, so every bf16 output is identical. The layer-1 input-projection
    class (K 1024, bias), a single 64-deep K-tile pair and a K that is not a power of two."""
    from two_towers_amd._lib import option
    dt = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(m + n + k)
    A = [torch.randn(m, k, generator=g, device=DEV).to(dt) for _ in range(nb)]
    B = [(torch.randn(n, k, generator=g, device=DEV) * k ** -0.5).to(dt) for _ in range(nb)]
    bias = [torch.randn(n, generator=g, device=DEV) for _ in range(nb)] if with_bias else None
    outs = []
    for w4 in (form, 0):
        C = [torch.full((m, n), float("nan"), device=DEV, dtype=dt) for _ in range(nb)]
        with option("gemm_w4", w4), option("gemm_bres", 0):
            ops.gemm(A, B, C, m=m, n=n, k=k, lda=k, ldb=k, ldc=n, a_kouter=False, b_kouter=False, dtype=dt,
                     out_dtype=dt, bias=bias, splits=1)
        torch.cuda.synchronize()
        outs.append(C)
    for i in range(nb):
        bad = int((outs[0][i].view(torch.int16) != outs[1][i].view(torch.int16)).sum())
        assert bad == 0, f"batch {i}: {bad} of {m * n} outputs differ"
    rows = torch.randint(0, m, (256,), generator=g, device=DEV)
    ref = A[0][rows].float() @ B[0].float().t() + (bias[0] if with_bias else 0)
    assert rel_err(outs[0][0][rows].float(), ref) < 8e-3


def test_gemm_input_projection_l1_class_hand_written():
    """The layer-1 input-projection class (bf16, both operands K-contiguous, K 1024,
    M >= 65536, bias, bf16 out; enhanced_two_tower.py:51,57 via nn.GRU layer 1) runs on the
    hand-written persistent kernel (no vendor GEMM is linked, include/tt_hip.h): against
    fp32 math on the bf16 operands, and run to run bit-identical (the training step is
    deterministic)."""
    from two_towers_amd._lib import option
    dt = torch.bfloat16
    m, n, k = 70144, 3072, 1024  # whole 256-row tiles: the interleaved-epilogue form (option gemm_iepi) applies
    g = torch.Generator(device=DEV).manual_seed(61)
    A = [torch.randn(m, k, generator=g, device=DEV).to(dt) for _ in range(2)]
    B = [(torch.randn(n, k, generator=g, device=DEV) * k ** -0.5).to(dt) for _ in range(2)]
    bias = [torch.randn(n, generator=g, device=DEV) for _ in range(2)]
    outs = []
    for _ in range(2):
        C = [torch.full((m, n), float("nan"), device=DEV, dtype=dt) for _ in range(2)]
        ops.gemm(A, B, C, m=m, n=n, k=k, lda=k, ldb=k, ldc=n, a_kouter=False, b_kouter=False, dtype=dt,
                 out_dtype=dt, bias=bias, splits=1)
        torch.cuda.synchronize()
        outs.append(C)
    # each tile's epilogue inside the next tile's first K-tile (gemm_iepi 1, the default) or
    # after its own last K-tile (0): the same values, bit for bit
    C0 = [torch.full((m, n), float("nan"), device=DEV, dtype=dt) for _ in range(2)]
    with option("gemm_iepi", 0):
        ops.gemm(A, B, C0, m=m, n=n, k=k, lda=k, ldb=k, ldc=n, a_kouter=False, b_kouter=False, dtype=dt,
                 out_dtype=dt, bias=bias, splits=1)
    torch.cuda.synchronize()
    rows = torch.randint(0, m, (1024,), generator=g, device=DEV)
    for i in range(2):
        assert torch.equal(outs[0][i], C0[i]), "interleaved and trailing epilogues differ"
        assert torch.equal(outs[0][i], outs[1][i]), "input projection not run-to-run identical"
        assert not torch.isnan(outs[0][i]).any()
        ref = A[i][rows].float() @ B[i].float().t() + bias[i]
        assert rel_err(outs[0][i][rows].float(), ref) < 8e-3


@pytest.mark.parametrize("m", [320, 296, 384, 400, 64])
@pytest.mark.parametrize("akout,bkout", [(1, 1), (0, 0)])
def test_gemm_tail_tile_idle_wave_row(m, akout, bkout):
    """256x256 tiles whose second wave row lies wholly past M (M mod 256 in (0, 128]) skip
    that row's MFMAs (tt_gemm_core.h Loop8::quad, mm = false): the layer-0 dW_ih^T shape
    (M = Ep 320, N = 3H, both operands K-outer, split-K, fp32 out) and ragged neighbours
    (tail 40, 128 exactly, 144: both rows live; M 64: one tile), against fp32 math."""
    dt = torch.bfloat16
    n, k = 1536, 8192
    g = torch.Generator().manual_seed(71 + m)
    A = torch.randn(m, k, generator=g).to(dt)
    B = torch.randn(n, k, generator=g).to(dt)
    Ad = (A.t().contiguous() if akout else A).to(DEV)
    Bd = (B.t().contiguous() if bkout else B).to(DEV)
    C = torch.full((m, n), float("nan"), device=DEV)
    ops.gemm([Ad], [Bd], [C], m=m, n=n, k=k, lda=m if akout else k, ldb=n if bkout else k, ldc=n,
             a_kouter=bool(akout), b_kouter=bool(bkout), dtype=dt, out_dtype=torch.float32)
    ref = A.float().to(DEV) @ B.float().to(DEV).t()
    assert not torch.isnan(C).any()
    assert rel_err(C, ref) < 1e-5, rel_err(C, ref)


@pytest.mark.parametrize("E,hidden", [(300, 256), (16, 8), (300, 512)])
def test_weight_pack_one_launch_matches_torch_pack(E, hidden):
    """towers._Packed's bf16 path (tt_pack_multi: stacked W_ih with layer 0 zero-padded to
    Ep, W_hh cast, r|z biases folded) against the torch path on the same parameters: every
    packed tensor bit-identical."""
    import two_towers_amd as tta
    from two_towers_amd import towers
    torch.manual_seed(E + hidden)
    m = tta.EnhancedTwoTowerModel(E, hidden).to(DEV)
    p = m._tower_params("query")
    H = 2 * hidden
    cfg = towers.TowerCfg(1, E, H, hidden, torch.bfloat16, 0.0)
    Ep = ops.pad_cols(E, torch.bfloat16)
    fast = towers._Packed(p, cfg, Ep)
    ref = towers._Packed.__new__(towers._Packed)
    ref.wih, ref.bias, ref.whh, ref.bhn = [], [], [], []
    ref._pack_torch(dict(zip(towers.GRU_NAMES, p[:16])), H, E, Ep, torch.bfloat16)
    torch.cuda.synchronize()
    for layer in (0, 1):
        assert torch.equal(fast.wih[layer], ref.wih[layer]), layer
        assert torch.equal(fast.bias[layer], ref.bias[layer]), layer
        for d in range(2):
            assert torch.equal(fast.whh[layer][d], ref.whh[layer][d]), (layer, d)
            assert torch.equal(fast.bhn[layer][d], ref.bhn[layer][d]), (layer, d)
