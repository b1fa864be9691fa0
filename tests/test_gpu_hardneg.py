"""tt_hardneg_topk (get_hard_negatives, enhanced_two_tower.py:123-133, batched) through the
C ABI. bf16 with h in {128, 256, 512} runs the streamed scan of tt_score.hip (chunk maxima ->
exact chunk selection -> bit-identical rescoring -> top-k); other shapes run the GEMM +
split top-k of tt_loss.hip. Integer-valued operands make every dot product exact in fp32
whatever the summation order, so indices -- ties included, which go to the lower column
-- and values are compared bit-exactly against a float64 reference of the reference rule
(positive column set to -1, then topk)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from two_towers_amd import _lib  # noqa: E402
from two_towers_amd._lib import call, dtype_code, option  # noqa: E402

DEV = "cuda"


def ref_hardneg(q, d, label_offset, k):
    s = (q.double() @ d.double().t()).cpu()
    if label_offset >= 0:
        rows = torch.arange(q.shape[0])
        s[rows, label_offset + rows] = -1.0
    # stable sort by (-value, index)
    order = torch.sort(-s, dim=1, stable=True).indices[:, :k]
    return order, torch.gather(s, 1, order)


def run_hardneg(q, d, label_offset, k, dt):
    lib = _lib.load()
    B, h = q.shape
    nd = d.shape[0]
    qd, dd = q.to(DEV, dt).contiguous(), d.to(DEV, dt).contiguous()
    idx = torch.empty(B, k, dtype=torch.int32, device=DEV)
    val = torch.empty(B, k, dtype=torch.float32, device=DEV)
    ws = torch.empty(max(lib.tt_hardneg_ws_size(dtype_code(dt), B, nd, h, k), 1), dtype=torch.uint8, device=DEV)
    call("tt_hardneg_topk", dtype_code(dt), qd.data_ptr(), B, dd.data_ptr(), nd, h, label_offset, k, idx.data_ptr(),
         val.data_ptr(), ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return idx.cpu().long(), val.cpu()


CASES = [  # B, nd, h, label_offset, k
    (300, 1000, 256, 0, 5),      # labels on the diagonal, nd not a multiple of 64
    (513, 513, 256, 0, 5),       # B = nd, partial row tile and partial chunk
    (64, 4096, 256, 1024, 5),    # label offset (DP rank 1 of 4)
    (257, 2000, 128, -1, 16),    # nothing masked (serving), k = 16
    (100, 200, 256, 0, 5),       # nch = 4 < k: every chunk selected
    (40, 70, 128, 3, 1),         # k = 1, two chunks
    (300, 1000, 512, 0, 5),      # h 512 (configs[4]): 4-wave scan, 2-slot ring
    (129, 4100, 512, 7, 16),     # h 512: partial row tile, odd tile count per split, k = 16
    (96, 640, 64, 0, 5),         # GEMM + split path (h = 64)
    (33, 999, 96, -1, 7),        # GEMM + split path (h = 96)
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,nd,h,lab,k", CASES)
def test_hardneg_exact(dt, B, nd, h, lab, k):
    g = torch.Generator().manual_seed(B * 7919 + nd * 31 + h)
    q = torch.randint(-3, 4, (B, h), generator=g).float()
    d = torch.randint(-3, 4, (nd, h), generator=g).float()
    d[nd // 2] = d[nd // 3]          # exact ties across chunks: lower index first
    d[nd - 1] = d[5]
    if nd > 130:
        d[70] = d[129]               # a tie inside neighbouring chunks
    ri, rv = ref_hardneg(q, d, lab, k)
    gi, gv = run_hardneg(q, d, lab, k, dt)
    assert torch.equal(gi, ri)
    assert torch.equal(gv.double(), rv)


@pytest.mark.parametrize("h", [128, 256, 512])
def test_hardneg_all_ties(h):
    """Every score equal: all chunk maxima tie, so the selection must take the lowest
    chunks and the result is the k lowest unmasked columns."""
    B, nd, k = 70, 900, 5
    q = torch.ones(B, h)
    d = torch.ones(nd, h)
    ri, rv = ref_hardneg(q, d, 0, k)
    gi, gv = run_hardneg(q, d, 0, k, torch.bfloat16)
    assert torch.equal(gi, ri)
    assert torch.equal(gv.double(), rv)


def test_hardneg_bench_size_consistent():
    """bench shape (8192 x 8192, h 256, bf16, normalised rows): the returned values are
    the float64 scores of the returned columns (to fp32 MFMA rounding), sorted, and no
    column outside the result scores more than the k-th result."""
    B, nd, h, k = 8192, 8192, 256, 5
    g = torch.Generator().manual_seed(11)
    q = torch.nn.functional.normalize(torch.randn(B, h, generator=g), dim=1).bfloat16().float()
    d = torch.nn.functional.normalize(torch.randn(nd, h, generator=g), dim=1).bfloat16().float()
    gi, gv = run_hardneg(q, d, 0, k, torch.bfloat16)
    s = (q.to(DEV).double() @ d.to(DEV).double().t())
    rows = torch.arange(B, device=DEV)
    s[rows, rows] = -1.0
    gi_d = gi.to(DEV)
    got = torch.gather(s, 1, gi_d)
    assert (got.cpu() - gv.double()).abs().max() < 1e-5
    assert bool((gv[:, :-1] >= gv[:, 1:]).all())
    s.scatter_(1, gi_d, -2.0)
    assert bool((s.max(dim=1).values.cpu() <= gv[:, -1].double() + 1e-5).all())
    assert len(set(gi[0].tolist())) == k


@pytest.mark.parametrize("B,nd,h,lab", [(1000, 3000, 256, 0), (300, 4100, 128, -1), (8192, 8192, 256, 0),
                                         (1000, 3000, 512, 0), (8192, 8192, 512, 0)])
def test_hardneg_scan_matches_gemm_path(B, nd, h, lab):
    """Random (non-integer) normalised bf16 rows: the streamed scan and the GEMM + split
    top-k path form every score with the same MFMA instruction and k order, so indices
    and values agree bit-exactly -- including near-ties, which a rescoring that differed
    from the scan's arithmetic by one ulp would flip."""
    g = torch.Generator().manual_seed(B + nd + h)
    q = torch.nn.functional.normalize(torch.randn(B, h, generator=g), dim=1)
    d = torch.nn.functional.normalize(torch.randn(nd, h, generator=g), dim=1)
    si, sv = run_hardneg(q, d, lab, 5, torch.bfloat16)
    with option("hn_gemm", 1):
        gi, gv = run_hardneg(q, d, lab, 5, torch.bfloat16)
    assert torch.equal(sv, gv)
    assert torch.equal(si, gi)


def _scan_with_cm(q, d, lab, k):
    """tt_hardneg_topk with the workspace kept: (idx, val, chunk maxima [B, nch])."""
    lib = _lib.load()
    B, h = q.shape
    nd = d.shape[0]
    dt = torch.bfloat16
    qd, dd = q.to(DEV, dt).contiguous(), d.to(DEV, dt).contiguous()
    idx = torch.empty(B, k, dtype=torch.int32, device=DEV)
    val = torch.empty(B, k, dtype=torch.float32, device=DEV)
    ws = torch.full((lib.tt_hardneg_ws_size(dtype_code(dt), B, nd, h, k),), 0x7F, dtype=torch.uint8, device=DEV)
    call("tt_hardneg_topk", dtype_code(dt), qd.data_ptr(), B, dd.data_ptr(), nd, h, lab, k, idx.data_ptr(),
         val.data_ptr(), ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    nch = (nd + 63) // 64
    return idx.cpu(), val.cpu(), ws[:B * nch * 4].view(torch.float32).view(B, nch).cpu()


@pytest.mark.parametrize("B,nd,h,lab,k", [(8192, 8192, 256, 0, 5), (1000, 3000, 256, 0, 5), (513, 513, 256, 0, 5),
                                          (300, 4100, 128, -1, 16), (64, 4096, 256, 1024, 5), (129, 4100, 512, 7, 16),
                                          (2048, 16384, 256, 100, 5), (40, 70, 128, 3, 1)])
def test_hardneg_scan_gemm_matches_scan_kernel(B, nd, h, lab, k):
    """The scan's chunk maxima from the persistent 256x256 GEMM with the chunk-max epilogue
    (option hn_scan_gemm 1: tt_gemm.hip gemm_persist HN; measured slower, not the default)
    against the streamed scan kernel (hn_scan_gemm 0, the default): the same MFMA instruction, operand orientation and k order,
    so every chunk maximum -- masked positive (-1) and tail columns (-inf) included -- and
    therefore every index and value is bit-identical. Ragged row tiles, partial chunks, label
    offsets, nothing masked, h 128 / 256 / 512, k 1 / 5 / 16."""
    g = torch.Generator().manual_seed(B + nd + h + k)
    q = torch.nn.functional.normalize(torch.randn(B, h, generator=g), dim=1)
    d = torch.nn.functional.normalize(torch.randn(nd, h, generator=g), dim=1)
    with option("hn_scan_gemm", 0):
        ki, kv, kcm = _scan_with_cm(q, d, lab, k)
    with option("hn_scan_gemm", 1):
        gi, gv, gcm = _scan_with_cm(q, d, lab, k)
    assert torch.equal(kcm.view(torch.int32), gcm.view(torch.int32)), int((kcm != gcm).sum())
    assert torch.equal(ki, gi) and torch.equal(kv, gv)
    ri, rv = ref_hardneg(q.to(torch.bfloat16).float(), d.to(torch.bfloat16).float(), lab, k)
    assert float((gv.double() - rv).abs().max()) < 1e-5  # fp32 accumulation of bf16 products


@pytest.mark.parametrize("B,nd,lab", [(8192, 8192, 0), (8192, 65536, 8192), (1000, 3000, 0), (513, 4100, 7),
                                      (40, 70, 3)])
def test_hardneg_scan_variants_match(B, nd, lab):
    """The h 256 scan's variants (option hn_scan_v: 5 the five-slot ring with the chunk maxima
    stored straight from registers, the default; 0 the round-3 form with the maxima staged in
    LDS; 4 64 queries per wave) under each block map: the same MFMA sequence per score, so the
    chunk maxima (masked positive and tail columns included) and the top-k are bit-identical.
    Shapes: the bench's 8192^2, the configs[3] per-rank pool (8192 x 65,536, labels at the
    rank's offset), ragged row tiles, partial chunks, fewer tiles than the ring's depth."""
    g = torch.Generator().manual_seed(B + nd + lab)
    q = torch.nn.functional.normalize(torch.randn(B, 256, generator=g), dim=1)
    d = torch.nn.functional.normalize(torch.randn(nd, 256, generator=g), dim=1)
    outs = {}
    with option("hn_scan_gemm", 0):
        for v in (5, 0, 4):
            for m in (0, 2):
                with option("hn_scan_v", v), option("hn_map", m):
                    outs[(v, m)] = _scan_with_cm(q, d, lab, 5)
    ri, rv, rcm = outs[(5, 2)]
    for key, (i, val, cm) in outs.items():
        assert torch.equal(rcm.view(torch.int32), cm.view(torch.int32)), (key, int((rcm != cm).sum()))
        assert torch.equal(ri, i) and torch.equal(rv, val), key


@pytest.mark.parametrize("B,nd,lab", [(8192, 8192, 0), (2048, 16384, 100), (1000, 3000, 0)])
@pytest.mark.parametrize("hn_map", [0, 1, 2])
def test_hardneg_scan_block_maps_agree(B, nd, lab, hn_map):
    """The scan's workgroup -> (row tile, document split) maps (option hn_map: 0 a split
    per XCD, 1 a row tile per XCD, 2 row-tile halves x split quarters per XCD, the default;
    2 falls back to 0 where the grid does not divide) only move work between workgroups:
    bit-identical."""
    g = torch.Generator().manual_seed(B + nd + hn_map)
    q = torch.nn.functional.normalize(torch.randn(B, 256, generator=g), dim=1)
    d = torch.nn.functional.normalize(torch.randn(nd, 256, generator=g), dim=1)
    with option("hn_scan_gemm", 0):  # the block maps are the scan kernel's
        si, sv = run_hardneg(q, d, lab, 5, torch.bfloat16)
        with option("hn_map", hn_map):
            mi, mv = run_hardneg(q, d, lab, 5, torch.bfloat16)
    assert torch.equal(sv, mv)
    assert torch.equal(si, mi)


def test_hardneg_hot_chunks():
    """Correlated rows (every query closest to the same few documents, as with a freshly
    initialised tower): all rows select the same chunks, so the rescoring of one chunk
    carries the whole batch."""
    B, nd, h, k = 4096, 4096, 256, 5
    g = torch.Generator().manual_seed(3)
    base = torch.randn(h, generator=g)
    q = torch.nn.functional.normalize(base + 0.05 * torch.randn(B, h, generator=g), dim=1).bfloat16().float()
    d = torch.nn.functional.normalize(torch.randn(nd, h, generator=g), dim=1)
    d[:64] = torch.nn.functional.normalize(base + 0.05 * torch.randn(64, h, generator=g), dim=1)
    d = d.bfloat16().float()
    si, sv = run_hardneg(q, d, 0, k, torch.bfloat16)
    with option("hn_gemm", 1):
        gi, gv = run_hardneg(q, d, 0, k, torch.bfloat16)
    assert torch.equal(sv, gv) and torch.equal(si, gi)
    assert bool((si < 64).all())


def ref_margin_grads(q, d, lab, idx, margin, gscale):
    q64, d64 = q.double().requires_grad_(True), d.double().requires_grad_(True)
    B, k = idx.shape
    pos = (q64 * d64[lab:lab + B]).sum(1)
    neg = (q64.unsqueeze(1) * d64[idx.long()]).sum(2).mean(1)
    loss = gscale * torch.clamp(margin - pos + neg, min=0).sum()
    loss.backward()
    return q64.grad, d64.grad


@pytest.mark.parametrize("B,nd,h,k,lab,hot", [(300, 900, 256, 5, 0, True), (1000, 1000, 256, 5, 0, False),
                                              (130, 700, 96, 16, 200, True), (64, 64, 1100, 3, 0, True),
                                              (50, 400, 64, 40, 100, True)])
def test_margin_bwd_repeated_negatives(B, nd, h, k, lab, hot):
    """tt_margin_bwd against float64 autograd of the reference rule
    (enhanced_two_tower.py:102-121 on normalised rows), with negatives repeated across
    rows (hot: a handful of documents mined by every row) or spread out. k = 40 takes
    16-row groups; two runs are bit-identical."""
    g = torch.Generator().manual_seed(B * 13 + k)
    q = torch.nn.functional.normalize(torch.randn(B, h, generator=g), dim=1)
    d = torch.nn.functional.normalize(torch.randn(nd, h, generator=g), dim=1)
    if hot:
        idx = torch.randint(0, 7, (B, k), generator=g, dtype=torch.int32) * 3
    else:
        idx = torch.randint(0, nd, (B, k), generator=g, dtype=torch.int32)
    margin, gscale = 2.0, 1.0 / B  # margin 2: every row active
    rq, rd = ref_margin_grads(q, d, lab, idx, margin, gscale)
    qd, dd, idd = q.to(DEV), d.to(DEV), idx.to(DEV)
    gdev = torch.tensor([gscale], dtype=torch.float32, device=DEV)  # device-side upstream gradient
    dq = torch.empty(B, h, device=DEV)
    outs = []
    for rep in range(2):  # deterministic: two runs give the same bits
        ddn = torch.zeros(nd, h, device=DEV)
        ws = torch.empty(_lib.load().tt_margin_bwd_ws_size(B, nd, h, k), dtype=torch.uint8, device=DEV)
        ws.fill_(0xA5 if rep else 0x5A)  # no result may depend on the workspace's previous contents
        call("tt_margin_bwd", qd.data_ptr(), B, dd.data_ptr(), nd, h, lab, idd.data_ptr(), k, margin, gdev.data_ptr(),
             dq.data_ptr(), ddn.data_ptr(), ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert (dq.cpu().double() - rq).abs().max() < 1e-6
        assert (ddn.cpu().double() - rd).abs().max() < 1e-5 * float(rd.abs().max()) + 1e-7
        outs.append(ddn.cpu())
    assert torch.equal(outs[0], outs[1])


def test_margin_bwd_requires_workspace():
    """The document gradient is summed through caller scratch: a null workspace is an
    argument error, not a silent fallback."""
    B, nd, h, k = 8, 16, 64, 2
    q = torch.zeros(B, h, device=DEV)
    d = torch.zeros(nd, h, device=DEV)
    idx = torch.zeros(B, k, dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError, match="workspace"):
        call("tt_margin_bwd", q.data_ptr(), B, d.data_ptr(), nd, h, 0, idx.data_ptr(), k, 0.2, None,
             q.data_ptr(), d.data_ptr(), None, torch.cuda.current_stream().cuda_stream)


# ---------------------------------------------------------------- configs[3] per-rank shape
# 8 ranks x 8192 pairs: every rank mines its 8192 queries against the all-gathered global
# pool of 65,536 documents, its own positives at columns rank * 8192 + i.

def test_hardneg_configs3_rank_shape_scan_matches_gemm_and_float64():
    """B_l 8192 x N 65,536 (rank 3 of 8), h 256, normalised bf16 rows: the streamed scan
    equals the GEMM + split top-k path bit for bit; against float64 (on the GPU) the
    returned values are the scores of the returned columns (to fp32 MFMA rounding),
    sorted, distinct, the positive is never returned and no other column scores above
    the k-th result."""
    B, nd, h, k, lab = 8192, 65536, 256, 5, 3 * 8192
    g = torch.Generator().manual_seed(81)
    q = torch.nn.functional.normalize(torch.randn(B, h, generator=g), dim=1).bfloat16().float()
    d = torch.nn.functional.normalize(torch.randn(nd, h, generator=g), dim=1).bfloat16().float()
    si, sv = run_hardneg(q, d, lab, k, torch.bfloat16)
    with option("hn_gemm", 1):
        gi, gv = run_hardneg(q, d, lab, k, torch.bfloat16)
    assert torch.equal(si, gi) and torch.equal(sv, gv)
    s = q.to(DEV).double() @ d.to(DEV).double().t()
    rows = torch.arange(B, device=DEV)
    s[rows, lab + rows] = -1.0
    gi_d = si.to(DEV)
    assert not bool((gi_d == (lab + rows)[:, None]).any())
    got = torch.gather(s, 1, gi_d)
    assert float((got.cpu() - sv.double()).abs().max()) < 1e-5
    assert bool((sv[:, :-1] >= sv[:, 1:]).all())
    assert all(len(set(r)) == k for r in si[:64].tolist())
    s.scatter_(1, gi_d, -2.0)
    assert bool((s.max(dim=1).values.cpu() <= sv[:, -1].double() + 1e-5).all())


def test_hardneg_configs3_pool_exact_with_ties():
    """1024 queries x the 65,536-row pool (label offset 5 * 1024), integer-valued rows so
    every score is exact: indices and values equal a stable float64 sort on the GPU,
    exact ties (copied documents far apart in the pool) going to the lower column."""
    B, nd, h, k, lab = 1024, 65536, 256, 5, 5 * 1024
    g = torch.Generator().manual_seed(82)
    q = torch.randint(-3, 4, (B, h), generator=g).float()
    d = torch.randint(-3, 4, (nd, h), generator=g).float()
    d[60000] = d[17]
    d[nd - 1] = d[40000]
    d[33000:33064] = d[100:164]
    gi, gv = run_hardneg(q, d, lab, k, torch.bfloat16)
    s = q.to(DEV).double() @ d.to(DEV).double().t()
    rows = torch.arange(B, device=DEV)
    s[rows, lab + rows] = -1.0
    ri = torch.sort(-s, dim=1, stable=True).indices[:, :k]
    rv = torch.gather(s, 1, ri)
    assert torch.equal(gi, ri.cpu())
    assert torch.equal(gv.double(), rv.cpu())
