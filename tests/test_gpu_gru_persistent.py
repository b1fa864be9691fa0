"""The persistent bf16 GRU forward (gru_fwd_seq, one launch per layer) against the
per-step forward (gru_fwd_step, option gru_step = 1) on every output it writes: the
layer output Y, the dropout copy X1 and the saved pre-activations S (r, z, n, gh_n).

Round 2 found the persistent kernel intermittently writing garbage into S's gh_n block
(step 0, lanes 12-15 of a 16-lane group). The cause was a hardware data hazard: a
16-byte buffer store whose soffset was an SGPR, followed at once by a VALU write of its
data registers, which LLVM leaves unprotected for that store form (DESIGN.md §3,
tools/check_store_hazard.py). These tests pin the fix at the bench grid (B 8192, T 64,
H 512, the four recurrences of configs[2]) and at the runtime-width instances (H 64 ..
448) that were retired because of it.

Reference: the recurrence of nn.GRU (enhanced_two_tower.py:17-33, called at :51, :57).
Both kernels run the same MFMA sequence along K and the same fp32 gate expression, so
every output is expected bit-identical; the fraction of differing elements and the
largest difference in bf16 ulps are printed.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

from two_towers_amd import _lib  # noqa: E402
from two_towers_amd._lib import GruFwdRec, call, option, stream_ptr  # noqa: E402
from two_towers_amd.towers import gru_fwd_workspace  # noqa: E402

DEV = "cuda"


def _inputs(ntow, B, T, H, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    G = [torch.randn(B * T, 6 * H, generator=g, device=DEV).to(torch.bfloat16) for _ in range(ntow)]
    whh = [[(torch.randn(3 * H, H, generator=g, device=DEV) * H ** -0.5).to(torch.bfloat16) for _ in range(2)]
           for _ in range(ntow)]
    bhn = [[torch.randn(H, generator=g, device=DEV) * 0.5 for _ in range(2)] for _ in range(ntow)]
    return G, whh, bhn


def _run(ntow, B, T, H, G, whh, bhn, drop_p, step, ws="auto"):
    """One tt_gru_fwd call; ws "auto": a zeroed workspace of tt_gru_fwd_ws_size bytes (the
    column-split kernel may run), None: no workspace (the row-owning kernel). Returns the
    launch count, the outputs and the workspace (its status word is ws[:4])."""
    dt = torch.bfloat16
    BT = B * T
    Y = [torch.empty(BT, 2 * H, dtype=dt, device=DEV) for _ in range(ntow)]
    X1 = [torch.empty(BT, 2 * H, dtype=dt, device=DEV) for _ in range(ntow)] if drop_p > 0 else None
    S = [[torch.empty(BT, 4 * H, dtype=dt, device=DEV) for _ in range(2)] for _ in range(ntow)]
    hs = torch.empty(ntow * 2, 2, B, H, dtype=torch.float32, device=DEV)
    recs = (GruFwdRec * (2 * ntow))()
    for ti in range(ntow):
        for d in range(2):
            r = recs[ti * 2 + d]
            r.g = G[ti][:, d * 3 * H:].data_ptr()
            r.whh = whh[ti][d].data_ptr()
            r.bhn = bhn[ti][d].data_ptr()
            r.y = Y[ti][:, d * H:].data_ptr()
            r.x1 = X1[ti][:, d * H:].data_ptr() if X1 is not None else None
            r.save = S[ti][d].data_ptr()
            r.hstate = hs[ti * 2 + d].data_ptr()
            r.dir = d
            r.drop_seed = 1234 + ti
            r.drop_col0 = d * H
            r.drop_row0 = 0
    with option("gru_step", step):
        if isinstance(ws, str):
            ws = gru_fwd_workspace(2 * ntow, B, T, H, dt, torch.device(DEV))
        launches = (_lib.load().tt_gru_fwd_launches_for(_lib.DT_BF16, 2 * ntow, B, T, H, 6 * H, 2 * H)
                    if ws is not None else _lib.load().tt_gru_fwd_launches(_lib.DT_BF16, T, H))
        call("tt_gru_fwd", _lib.DT_BF16, recs, 2 * ntow, B, T, H, 6 * H, 2 * H, drop_p,
             ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0, stream_ptr())
        torch.cuda.synchronize()
    return launches, Y, X1, S, ws


def _status(ws):
    return 0 if ws is None else int(ws[:4].view(torch.int32).item())


def _ulps(a, b):
    """Largest distance in bf16 ulps between two bf16 tensors (same-sign ordering)."""
    ia = a.view(torch.int16).to(torch.int32)
    ib = b.view(torch.int16).to(torch.int32)
    # map sign-magnitude to a monotone integer line
    ia = torch.where(ia < 0, -(ia & 0x7FFF), ia)
    ib = torch.where(ib < 0, -(ib & 0x7FFF), ib)
    return int((ia - ib).abs().max().item())


def _compare(name, a, b, stats):
    ne = int((a.view(torch.int16) != b.view(torch.int16)).sum().item())
    u = _ulps(a, b) if ne else 0
    stats.append((name, ne, a.numel(), u))
    return ne, u


def _check_step0_ghn(S, bhn, B, T, H):
    """At a recurrence's first step h_{-1} = 0, so the saved gh_n = W_hn h + b_hn is
    exactly bf16(b_hn) in every row: the slot the round-2 corruption hit."""
    for ti in range(len(S)):
        for d in range(2):
            t0 = 0 if d == 0 else T - 1
            ghn = S[ti][d].view(B, T, 4 * H)[:, t0, 3 * H:]
            want = bhn[ti][d].to(torch.bfloat16).expand(B, H)
            bad = int((ghn.view(torch.int16) != want.view(torch.int16)).sum().item())
            assert bad == 0, f"tower {ti} dir {d}: {bad} corrupted gh_n values at step 0"


def _assert_equivalent(outs_p, outs_s, B, T, H, bhn):
    lp, Yp, X1p, Sp, wsp = outs_p
    ls, Ys, X1s, Ss, _ = outs_s
    assert _status(wsp) == 0, "a column-split member wait timed out"
    assert lp == 1 and ls == T, (lp, ls)
    stats = []
    for ti in range(len(Yp)):
        _compare(f"Y{ti}", Yp[ti], Ys[ti], stats)
        if X1p is not None:
            _compare(f"X1{ti}", X1p[ti], X1s[ti], stats)
        for d in range(2):
            for gi, gname in enumerate(("r", "z", "n", "ghn")):
                _compare(f"S{ti}{d}.{gname}", Sp[ti][d][:, gi * H:(gi + 1) * H], Ss[ti][d][:, gi * H:(gi + 1) * H],
                         stats)
    for name, ne, n, u in stats:
        print(f"{name}: {ne} of {n} differ, max {u} ulp")
    for ti in range(len(Sp)):
        for d in range(2):
            assert torch.isfinite(Sp[ti][d].float()).all()
            assert float(Sp[ti][d].float().abs().max()) < 1e3
    _check_step0_ghn(Sp, bhn, B, T, H)
    _check_step0_ghn(Ss, bhn, B, T, H)
    bad = [(name, ne, u) for name, ne, n, u in stats if ne]
    assert not bad, f"persistent vs per-step forward differ: {bad}"


@pytest.mark.parametrize("xc,xs", [(0, 1), (1, 1), (1, 0)])
def test_bench_grid_persistent_forward_matches_per_step(xc, xs):
    """configs[2] layer-0 shape: B 8192, T 64, H 512, 2 towers x 2 directions in one
    launch, dropout 0.1 on the X1 copy: the persistent forward (xc 1: the column-split
    forward the bench runs, xs 1 its matrix/vector-wave form gru_fwd_xs, xs 0 the
    single-role gru_fwd_xcp; xc 0: the row-owning gru_fwd_seq<4,8>) vs T launches of
    gru_fwd_step."""
    B, T, H, ntow = 8192, 64, 512, 2
    G, whh, bhn = _inputs(ntow, B, T, H, seed=3)
    outs_s = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=1)
    with option("gru_fwd_xc", xc), option("gru_fwd_xs", xs):
        outs_p = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=0)
    assert (outs_p[4] is not None) == (xc == 1)
    _assert_equivalent(outs_p, outs_s, B, T, H, bhn)


@pytest.mark.parametrize("H,B,T,ntow", [(512, 1000, 12, 2), (256, 1000, 12, 2), (512, 3000, 5, 2), (512, 70, 3, 2),
                                        (256, 64, 1, 2), (512, 5000, 7, 1), (256, 8192, 4, 2), (512, 300, 2, 1)])
def test_column_split_forward_matches_per_step(H, B, T, ntow):
    """The column-split forward forced (option gru_fwd_xc = 2) wherever it applies: the H/64 member
    workgroups of a group exchange h every step through the caller's workspace. Rows per
    group that are not a multiple of the 256-row round (B 3000 over 8 groups per
    recurrence: 375 = 256 + 119), groups with no rows at all (B 70, B 64), one tower
    (two recurrences: 16 groups each) and T = 1; same MFMA k order and gate arithmetic as
    the per-step kernel, so every output is bit-identical."""
    G, whh, bhn = _inputs(ntow, B, T, H, seed=11 * H + B + T + ntow)
    outs_s = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=1)
    # 2: images kept in the XCD's L2 where a group shares one (the usual placement);
    # 6: every image store write-through; 18 / 22: a group's members are consecutive blocks,
    # i.e. dealt over the 8 XCDs, so the exchange really crosses XCD L2s (the members see
    # different XCC ids and take the write-through hand-off; 18 checks that they do)
    # H 512 runs both forms: gru_fwd_xs (matrix / vector waves, the default) and gru_fwd_xcp
    for xs in ((1, 0) if H == 512 else (1,)):
        for mode in (2, 6, 18, 22):
            with option("gru_fwd_xc", mode), option("gru_fwd_xs", xs):
                outs_p = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=0)
            assert outs_p[0] == 1 and outs_p[4] is not None, (xs, mode)
            _assert_equivalent(outs_p, outs_s, B, T, H, bhn)


def test_column_split_forward_without_workspace_runs_row_owning_kernel():
    """No workspace (or one smaller than tt_gru_fwd_ws_size): tt_gru_fwd runs the row-owning
    gru_fwd_seq instead -- the kernels never allocate; outputs equal the per-step kernel's."""
    B, T, H, ntow = 2048, 6, 512, 2
    G, whh, bhn = _inputs(ntow, B, T, H, seed=5)
    lib = _lib.load()
    assert lib.tt_gru_fwd_ws_size(_lib.DT_BF16, 4, B, T, H, 6 * H, 2 * H) > 0
    assert lib.tt_gru_fwd_ws_size(_lib.DT_F32, 4, B, T, H, 6 * H, 2 * H) == 0
    assert lib.tt_gru_fwd_ws_size(_lib.DT_BF16, 4, B, T, 1024, 6 * 1024, 2 * 1024) == 0
    outs_s = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=1)
    _assert_equivalent(_run(ntow, B, T, H, G, whh, bhn, 0.1, step=0, ws=None), outs_s, B, T, H, bhn)
    small = torch.zeros(256, dtype=torch.uint8, device=DEV)
    _assert_equivalent(_run(ntow, B, T, H, G, whh, bhn, 0.1, step=0, ws=small), outs_s, B, T, H, bhn)


def test_column_split_member_timeout_is_reported_and_not_sticky():
    """A member that never publishes (diagnostic option gru_xc_skip) makes the other
    members' waits give up (bound lowered with gru_xc_spins): the launch sets the caller's
    status word -- and the model path raises GruTimeoutError from check_gru_status instead
    of training on the invalid outputs. The per-launch flag lives with the counters, so
    the next launch on a fresh workspace is valid and bit-identical again."""
    import two_towers_amd as tta
    B, T, H, ntow = 2048, 4, 512, 2
    G, whh, bhn = _inputs(ntow, B, T, H, seed=9)
    outs_s = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=1)
    with option("gru_xc_spins", 14), option("gru_xc_skip", 3):
        bad = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=0)
    assert bad[0] == 1 and _status(bad[4]) != 0
    _assert_equivalent(_run(ntow, B, T, H, G, whh, bhn, 0.1, step=0), outs_s, B, T, H, bhn)
    # the nn.Module path: the next forward (or an explicit check) raises
    torch.manual_seed(0)
    m = tta.EnhancedTwoTowerModel(40, H // 2).to(DEV).set_compute_dtype(torch.bfloat16).train()
    q = torch.randn(B, T, 40, device=DEV)
    tta.check_gru_status()
    with option("gru_xc_spins", 14), option("gru_xc_skip", 1):
        m(q, q)
    with pytest.raises(tta.GruTimeoutError):
        tta.check_gru_status()
    m(q, q)  # healthy again
    tta.check_gru_status()
    # contained on the device: a timed-out forward's backward and Adam step leave every
    # parameter and moment bit-unchanged (the step guard), although the host learns of the
    # timeout only afterwards; the next healthy step trains normally
    opt = tta.Adam(m.parameters(), lr=1e-2)
    crit = tta.InfoNCELoss()
    crit(*m(q, q)).backward()
    opt.step()  # one healthy step, so the moments are non-zero
    opt.zero_grad()
    tta.check_gru_status()
    # the guard the first timed-out forward armed was cleared once the host had been told of
    # it (the raise above), so this step trained
    for p in m.parameters():
        assert opt.state[p]["exp_avg_sq"].abs().sum() > 0
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    moments = {id(p): (opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone()) for p in m.parameters()}
    with option("gru_xc_spins", 14), option("gru_xc_skip", 1):
        vq, vd = m(q, q)
    # the host-side check of TowersFn.backward (wait=False) would raise already when the
    # forward has finished; switched off here so the step runs as it does when the host is
    # still ahead of the GPU -- the case only the device-side guard covers
    from two_towers_amd import towers
    host_check = towers.check_gru_status
    towers.check_gru_status = lambda wait=True: None
    try:
        crit(vq, vd).backward()
        opt.step()
    finally:
        towers.check_gru_status = host_check
    torch.cuda.synchronize()
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k]), k
    for p in m.parameters():
        assert torch.equal(opt.state[p]["exp_avg"], moments[id(p)][0])
        assert torch.equal(opt.state[p]["exp_avg_sq"], moments[id(p)][1])
    with pytest.raises(tta.GruTimeoutError):
        tta.check_gru_status()
    opt.zero_grad()
    crit(*m(q, q)).backward()
    opt.step()
    tta.check_gru_status()
    assert any(not torch.equal(v, before[k]) for k, v in m.state_dict().items())
    # the skipped step is not counted: two applied updates
    opt.settle_skipped_steps()
    assert all(int(opt.state[p]["step"]) == 2 for p in m.parameters())
    # an eval / no-grad forward that times out does not arm the guard
    with torch.no_grad(), option("gru_xc_spins", 14), option("gru_xc_skip", 1):
        m(q, q)
    with pytest.raises(tta.GruTimeoutError):
        tta.check_gru_status()
    snap = {k: v.detach().clone() for k, v in m.state_dict().items()}
    opt.zero_grad()
    crit(*m(q, q)).backward()
    opt.step()
    torch.cuda.synchronize()
    assert any(not torch.equal(v, snap[k]) for k, v in m.state_dict().items())


def test_column_split_forward_beside_a_busy_stream_is_valid_or_reported():
    """The column-split forward is a plain launch by default (option gru_xc_coop 0): the
    occupancy query proves only that the grid fits an idle device, so kernels on another
    stream can keep members from being co-resident. Then either the members still meet (the
    other work drains first) and every output is bit-identical to the quiet-device run, or a
    bounded wait gives up and the launch reports it in its status word -- never wrong outputs
    silently (the status reaches the host as GruTimeoutError and the optimiser's step guard).
    Here torch GEMMs fill every CU from a second stream while the forward is launched."""
    B, T, H, ntow = 8192, 8, 512, 2
    G, whh, bhn = _inputs(ntow, B, T, H, seed=21)
    ref = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=1)  # per-step kernel: the bit-identical reference
    a = torch.randn(8192, 8192, device=DEV).to(torch.bfloat16)
    hog, fwd = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(hog):
        for _ in range(12):
            c = a @ a  # ~1 ms each on every CU
    with torch.cuda.stream(fwd):
        out = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=0)
    torch.cuda.synchronize()
    del c
    st = _status(out[4])
    print(f"forward beside a busy stream: status {st}")
    if st == 0:
        _assert_equivalent(out, ref, B, T, H, bhn)


@pytest.mark.parametrize("H,depth", [(64, 4), (128, 4), (128, 1), (192, 4), (256, 2), (320, 4), (384, 4), (448, 4),
                                     (512, 1)])
def test_runtime_width_persistent_forward_matches_per_step(H, depth):
    """The runtime-K-tile-count instances (gru_fwd_seq<D,0>: every H % 64 == 0 below 512
    other than 256) and a fixed one per register-ring depth D (option gru_depth), with a
    tail workgroup (B = 1000 = 15 x 64 + 40) and dropout on."""
    B, T, ntow = 1000, 12, 2
    G, whh, bhn = _inputs(ntow, B, T, H, seed=H + depth)
    outs_s = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=1)
    with option("gru_depth", depth):
        outs_p = _run(ntow, B, T, H, G, whh, bhn, 0.1, step=0)
    _assert_equivalent(outs_p, outs_s, B, T, H, bhn)
