"""Forward/backward of one or two encoder towers on the HIP path.

A tower is the reference's encoder: nn.GRU(E, 2h, num_layers=2, bidirectional,
dropout=0.1) followed by Linear(4h,2h) -> LayerNorm -> ReLU -> Linear(2h,h)
(enhanced_two_tower.py:17-48, :50-60). The query and doc towers of
EnhancedTwoTowerModel.forward (:62-65) run through the same kernel launches: every
GEMM is batched over towers (and directions) and every GRU step launch covers all
four recurrences.

Layout in HBM (per tower; row = b*T + t, dt = compute dtype):
  X0  [B*T, Ep]  dt   layer-0 input (gathered Word2Vec rows / packed floats)
  G   [B*T, 6H]  dt   input projections, fwd gates r|z|n then rev gates
  Y   [B*T, 2H]  dt   layer output h_t (fwd | rev), X1 = dropout(Y0) (layer-1 input)
  S   [B*T, 4H]  dt   saved pre-activations of r|z|n and gh_n per direction
  dG  [B*T, 8H]  dt   gradients wrt gate pre-activations: dL/dg_x r|z|n (fwd, rev) in
                      [0, 6H), dL/d(W_hn h) (fwd, rev) in [6H, 8H); dL/dg_h shares r|z
"""
from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from . import _lib, dist, ops, timing
from ._lib import GruBwdRec, GruFwdRec, HeadBwdIO, HeadFwdIO, call, dtype_code, stream_ptr

PARAMS_PER_TOWER = 22
LN_EPS = 1e-5
HEAD_DT = torch.float32


def gru_param_names():
    names = []
    for layer in (0, 1):
        for sfx in ("", "_reverse"):
            for w in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
                names.append(f"{w}_l{layer}{sfx}")
    return names


GRU_NAMES = gru_param_names()
HEAD_NAMES = ["0.weight", "0.bias", "1.weight", "1.bias", "3.weight", "3.bias"]


@dataclass(frozen=True)
class TowerCfg:
    ntowers: int
    E: int
    H: int  # GRU hidden per direction (= 2 * hidden_dim)
    h: int  # output dim (= hidden_dim)
    dtype: torch.dtype
    drop_p: float  # dropout between GRU layers (0 in eval)
    head: str = "proj2"  # "proj2": per-tower enhanced head; "none": return cat(h_fwd, h_rev) [B, 2H]
    rank: int = 0  # data-parallel rank: dropout mask rows start at rank * B * T (global batch rows)

    @property
    def nparams(self) -> int:
        return PARAMS_PER_TOWER if self.head == "proj2" else len(GRU_NAMES)


_PACK_ONE = os.environ.get("TT_PACK_TORCH", "0") == "0"  # 0: bf16 packs in one launch (read once)


class _Packed:
    """Per-step compute-dtype copies of one tower's weights in the kernels' layouts."""

    def __init__(self, p, cfg: TowerCfg, Ep: int):
        dt, H, E = cfg.dtype, cfg.H, cfg.E
        g = dict(zip(GRU_NAMES, p[:16]))
        hd = dict(zip(HEAD_NAMES, p[16:]))
        self.wih = []
        self.bias = []
        self.whh = []
        self.bhn = []
        if _PACK_ONE and dt == torch.bfloat16 and E % 4 == 0 and H % 4 == 0 and all(
                t.is_contiguous() and t.dtype == torch.float32 and t.data_ptr() % 16 == 0 for t in p[:16]):
            self._pack_bf16(g, H, E, Ep, p[0].device)
        else:
            self._pack_torch(g, H, E, Ep, dt)
        if cfg.head == "none":
            return
        # The projection head always runs in fp32 (HEAD_DT): it is <1% of the FLOPs, and its
        # backward is where the batch-wide cancellation of the contrastive-loss gradient
        # would otherwise lose most of its precision to a bf16 cast.
        self.w1 = hd["0.weight"].float().contiguous()
        self.b1 = hd["0.bias"].float().contiguous()
        self.ln_g = hd["1.weight"].float().contiguous()
        self.ln_b = hd["1.bias"].float().contiguous()
        self.w2 = hd["3.weight"].float().contiguous()
        self.b2 = hd["3.bias"].float().contiguous()

    def _pack_bf16(self, g, H, E, Ep, dev):
        """The bf16 packs in one launch (tt_pack_multi): W_ih of both directions stacked
        (layer 0 zero-padded to Ep columns), W_hh cast, biases with the r|z parts of b_hh
        folded in -- the same values as _pack_torch (fp32 adds, round-to-nearest-even)."""
        jobs = (_lib.PackJob * 16)()
        nj = 0

        def job(src, dst, rows, cols, dcols, lds, ldd, bf16, src2=None):
            nonlocal nj
            j = jobs[nj]
            j.src, j.src2, j.dst = src, src2, dst
            j.rows, j.cols, j.dcols, j.lds, j.ldd, j.dst_bf16 = rows, cols, dcols, lds, ldd, int(bf16)
            nj += 1
        for layer in (0, 1):
            K = E if layer == 0 else 2 * H
            Kp = Ep if layer == 0 else K
            w = _alloc((6 * H, Kp), torch.bfloat16, dev)
            b = _alloc((6 * H,), torch.float32, dev)
            whh = []
            for d, sfx in enumerate(("", "_reverse")):
                job(g[f"weight_ih_l{layer}{sfx}"].data_ptr(), w.data_ptr() + d * 3 * H * Kp * 2, 3 * H, K, Kp, K, Kp, True)
                bi, bh = g[f"bias_ih_l{layer}{sfx}"], g[f"bias_hh_l{layer}{sfx}"]
                job(bi.data_ptr(), b.data_ptr() + d * 3 * H * 4, 1, 2 * H, 2 * H, 2 * H, 2 * H, False, bh.data_ptr())
                job(bi.data_ptr() + 2 * H * 4, b.data_ptr() + (d * 3 + 2) * H * 4, 1, H, H, H, H, False)
                wh = _alloc((3 * H, H), torch.bfloat16, dev)
                job(g[f"weight_hh_l{layer}{sfx}"].data_ptr(), wh.data_ptr(), 3 * H, H, H, H, H, True)
                whh.append(wh)
            self.wih.append(w)
            self.bias.append(b)
            self.whh.append(whh)
            self.bhn.append([g[f"bias_hh_l{layer}{s}"][2 * H:] for s in ("", "_reverse")])
        call("tt_pack_multi", jobs, nj, stream_ptr(dev))

    def _pack_torch(self, g, H, E, Ep, dt):
        for layer in (0, 1):
            wf, wr = g[f"weight_ih_l{layer}"], g[f"weight_ih_l{layer}_reverse"]
            w = torch.cat([wf, wr], 0)
            if layer == 0 and Ep != E:
                w = F.pad(w, (0, Ep - E))
            self.wih.append(w.to(dt).contiguous())
            bs = []
            for sfx in ("", "_reverse"):
                bi, bh = g[f"bias_ih_l{layer}{sfx}"], g[f"bias_hh_l{layer}{sfx}"]
                bs.append(torch.cat([bi[: 2 * H] + bh[: 2 * H], bi[2 * H:]]))
            self.bias.append(torch.cat(bs).float().contiguous())
            self.whh.append([g[f"weight_hh_l{layer}{s}"].to(dt).contiguous() for s in ("", "_reverse")])
            self.bhn.append([g[f"bias_hh_l{layer}{s}"][2 * H:].float().contiguous() for s in ("", "_reverse")])


def _packed(p, cfg: TowerCfg, Ep: int, cache_ok: bool) -> _Packed:
    """_Packed of one tower's parameters; for inference calls, cached on the first
    parameter and reused while every parameter keeps its autograd version and storage
    (optimizer steps and load_state_dict bump the version; two_towers_amd.Adam bumps it
    explicitly). Writes through `.data` bypass version tracking, as for autograd itself."""
    if not cache_ok:
        return _Packed(p, cfg, Ep)
    key = (cfg.dtype, cfg.H, cfg.head, Ep, tuple(t._version for t in p), tuple(t.data_ptr() for t in p))
    hit = getattr(p[0], "_tt_pack", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    pk = _Packed(p, cfg, Ep)
    p[0]._tt_pack = (key, pk)
    return pk


def _alloc(shape, dt, dev):
    return torch.empty(shape, dtype=dt, device=dev)


# ---- column-split GRU forward: caller-owned workspace and its status word --------------
# tt_gru_fwd runs the column-split kernel (member workgroups that exchange h every step)
# only with a workspace from the caller (include/tt_hip.h tt_gru_fwd_ws_size). Its first
# word is a status the kernels set when a member wait timed out -- the launch's outputs
# are then invalid. Two things follow from it, neither of which synchronises the host:
#  * on the device, the word is OR-ed into a per-device step guard; two_towers_amd.Adam
#    passes the guard to tt_adam_multi, which then leaves every parameter and moment
#    unchanged, and clears it after the step -- an invalid forward can never update the
#    weights, whatever the host has not yet seen;
#  * on the host, the word is copied to pinned memory on the stream; check_gru_status()
#    raises GruTimeoutError for any such launch. TowersFn.forward checks every earlier
#    forward (waiting on its event: the host is at most the GPU's queue ahead, which still
#    holds later work, so the GPU never idles for it), TowersFn.backward the ones already
#    finished.
# The guard is armed only by forwards that record autograd state (an eval / no-grad forward
# feeds no optimiser step), and once check_gru_status has reported a timeout to the host the
# guard of that device is cleared, stream-ordered, by the next forward: from then on the host
# owns the recovery, and a healthy step after it trains. two_towers_amd.Adam does not count a
# step the device skipped (it reads each step's guard back asynchronously and takes the step
# off the parameters' step counters at its next call).
_status_lock = threading.Lock()
_status_pending: list = []  # (event, pinned int32[1], device)
_step_guard: dict = {}  # device -> int32[1]: OR of the status words since the last optimiser step
_guard_reset: set = set()  # devices whose timeout the host has been told of: cleared at the next forward


def step_guard(dev) -> torch.Tensor:
    """The device's step-guard word (int32[1]; non-zero: a forward since the last optimiser
    step timed out)."""
    dev = torch.device(dev)
    with _status_lock:
        g = _step_guard.get(dev)
        if g is None:
            g = _step_guard[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
    return g


def gru_fwd_workspace(nrec, B, T, H, dt, dev):
    """Zero-status workspace for one tt_gru_fwd call shape, or None when the column-split
    kernel does not apply (tt_gru_fwd then runs the row-owning kernel without one)."""
    nb = _lib.load().tt_gru_fwd_ws_size(dtype_code(dt), nrec, B, T, H, 6 * H, 2 * H)
    if nb <= 0:
        return None
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    if ws.data_ptr() % 256:
        raise _lib.TTError("GRU forward workspace is not 256-byte aligned")
    ws[:256].zero_()
    return ws


def reset_guard_if_reported(dev):
    """Before a forward's launches: clear the device's step guard (stream-ordered) if the host
    has been told of a timed-out forward since the guard was last cleared."""
    dev = torch.device(dev)
    with _status_lock:
        due = dev in _guard_reset
        _guard_reset.discard(dev)
    if due:
        with torch.cuda.device(dev):
            step_guard(dev).zero_()


def watch_gru_status(ws, arm: bool = True):
    """After the launches using ws (on its device's current stream): fold its status word
    into the device's step guard (arm: the forward records autograd state, so an optimiser
    step may follow) and queue an asynchronous read-back for the host."""
    with torch.cuda.device(ws.device):
        st = torch.cuda.current_stream(ws.device)
        word = ws[:4].view(torch.int32)
        if arm:
            step_guard(ws.device).bitwise_or_(word)
        host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        host.copy_(word, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(st)
    with _status_lock:
        _status_pending.append((ev, host, torch.device(ws.device)))


def check_gru_status(wait: bool = True):
    """Raise GruTimeoutError if a watched column-split forward gave up a member wait.
    wait=False checks only the launches that have already finished."""
    with _status_lock:
        pend = list(_status_pending)
        _status_pending.clear()
    bad = 0
    keep = []
    bad_devs = set()
    for ev, host, dev in pend:
        if not wait and not ev.query():
            keep.append((ev, host, dev))
            continue
        ev.synchronize()
        if host.item() != 0:
            bad += 1
            bad_devs.add(dev)
    with _status_lock:
        if keep:
            _status_pending[:0] = keep
        _guard_reset.update(bad_devs)
    if bad:
        raise _lib.GruTimeoutError(
            f"{bad} column-split GRU forward launch(es) timed out waiting for a member workgroup "
            "(not all workgroups were resident); their outputs are invalid and the optimiser step "
            "that followed (two_towers_amd.Adam) left the weights unchanged. Set option gru_fwd_xc=0 "
            "(env TT_GRU_FWD_XC=0) to use the row-owning kernel.")


def _xs_selected() -> bool:
    """Whether tt_gru_fwd's column-split form is gru_fwd_xs (option gru_fwd_xs; a library
    without the option runs gru_fwd_xcp)."""
    try:
        return bool(_lib.get_option("gru_fwd_xs"))
    except _lib.TTError:
        return False


def table_cols(table, x):
    return getattr(table, "real_cols", table.shape[1])


def featurize(x: torch.Tensor, table: torch.Tensor | None, Ep: int, dt: torch.dtype) -> torch.Tensor:
    """[B,T] ids -> gathered rows, or [B,T,E] floats -> packed rows; returns [B*T, Ep]."""
    if x.dtype in (torch.int32, torch.int64):
        if table is None:
            raise _lib.TTError("integer token ids need an embedding table (model.set_embedding_table)")
        if table.dtype != dt or table.shape[1] != Ep:
            raise _lib.TTError(f"embedding table must be {dt} with {Ep} columns, got {table.dtype} {tuple(table.shape)}")
        ids = x.reshape(-1).to(torch.int32).contiguous()
        out = _alloc((ids.numel(), Ep), dt, x.device)
        esz = 2 if dt == torch.bfloat16 else 4
        # algorithmic bytes per row: id + the E real columns read and written
        gb = ids.numel() * (4 + 2 * table_cols(table, x) * esz)
        with timing.region("embed_gather", 1, gb, gb):
            ops.embed_gather(table, ids, out)
        return out
    if x.dim() != 3:
        raise ValueError(f"expected [B, T, E] embeddings or [B, T] token ids, got shape {tuple(x.shape)}")
    src = x.float().contiguous()
    out = _alloc((src.shape[0] * src.shape[1], Ep), dt, x.device)
    ops.pack_rows(src, out)
    return out


def _gru_layer_fwd(cfg, xs, K, ldx, packs, layer, B, T, seeds, want_x1, ws):
    """Input projection + one bidirectional GRU layer for every tower. The dropout copy
    X1 (want_x1) draws keep(seed, rank*B*T + b*T + t, col): on N data-parallel ranks the
    masks are those the single-process run of the global batch draws."""
    n, H, dt, dev = cfg.ntowers, cfg.H, cfg.dtype, xs[0].device
    BT = B * T
    G = [_alloc((BT, 6 * H), dt, dev) for _ in range(n)]
    esz = 2 if dt == torch.bfloat16 else 4
    kr = cfg.E if layer == 0 else K  # algorithmic work counts the real columns, not the padding
    with timing.region(f"input_proj_l{layer}", 1, 2.0 * BT * 6 * H * kr * n,
                       float(n * esz * (BT * kr + 6 * H * kr + BT * 6 * H))):
        ops.gemm(xs, [p.wih[layer] for p in packs], G, m=BT, n=6 * H, k=K, lda=ldx, ldb=K, ldc=6 * H,
                 a_kouter=False, b_kouter=False, dtype=dt, out_dtype=dt, bias=[p.bias[layer] for p in packs])
    Y = [_alloc((BT, 2 * H), dt, dev) for _ in range(n)]
    X1 = [_alloc((BT, 2 * H), dt, dev) for _ in range(n)] if want_x1 else None
    S = [[_alloc((BT, 4 * H), dt, dev) for _ in range(2)] for _ in range(n)]
    hs = _alloc((n * 2, 2, B, H), torch.float32, dev)
    recs = (GruFwdRec * (2 * n))()
    for ti in range(n):
        for d in range(2):
            r = recs[ti * 2 + d]
            r.g = G[ti][:, d * 3 * H:].data_ptr()
            r.whh = packs[ti].whh[layer][d].data_ptr()
            r.bhn = packs[ti].bhn[layer][d].data_ptr()
            r.y = Y[ti][:, d * H:].data_ptr()
            r.x1 = X1[ti][:, d * H:].data_ptr() if want_x1 else None
            r.save = S[ti][d].data_ptr()
            r.hstate = hs[ti * 2 + d].data_ptr()
            r.dir = d
            r.drop_seed = seeds[ti] & 0xFFFFFFFF
            r.drop_col0 = d * H
            r.drop_row0 = (cfg.rank * B * T) & 0xFFFFFFFF
    # algorithmic bytes per (row, unit, step): gates 3 + h 1 + saved 4 (+ dropout copy 1)
    # elements of dt; the per-step kernel also re-reads h_{s-1} (1 element) and moves the
    # fp32 recurrent state through HBM (8 B), the persistent one keeps both on chip
    nl = _lib.load().tt_gru_fwd_launches_for(dtype_code(dt), 2 * n, B, T, H, 6 * H, 2 * H) if ws is not None \
        else _lib.load().tt_gru_fwd_launches(dtype_code(dt), T, H)
    per = esz * (8 + (1 if want_x1 else 0)) + (0 if nl == 1 else esz + 8)
    if nl == 1 and ws is not None:
        form = "gru_fwd_xs" if H == 512 and _xs_selected() else "gru_fwd_xcp"
        kname = f"{form}<{H}, {'true' if want_x1 and cfg.drop_p > 0 else 'false'}>"
    elif nl == 1:
        kname = "gru_fwd_seq<"
    else:
        kname = "gru_fwd_step<"
    with timing.region("gru_fwd", nl, 2.0 * B * H * 3 * H * 2 * n * (T - 1), float(B * T * H * 2 * n * per),
                       kernel=kname):
        call("tt_gru_fwd", dtype_code(dt), recs, 2 * n, B, T, H, 6 * H, 2 * H, cfg.drop_p if want_x1 else 0.0,
             ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0, stream_ptr(dev))
    del G
    return Y, X1, S


def _gru_layer_bwd(cfg, layer, B, T, S, Y, dY, dfinal, packs):
    """Returns dG ([B*T, 8H] per tower: dL/dg_x of both directions in columns [0, 6H),
    dL/d(W_hn h) of both directions in [6H, 8H); dL/dg_h = [r|z of dL/dg_x, W_hn block])
    and bias grads (dbih, dbhh per tower/dir)."""
    n, H, dt, dev = cfg.ntowers, cfg.H, cfg.dtype, Y[0].device
    BT = B * T
    lib = _lib.load()
    dG = [_alloc((BT, 8 * H), dt, dev) for _ in range(n)]
    dhs = _alloc((n * 2, 2, B, H), dt, dev)
    nbr = lib.tt_gru_bias_rows(B)
    part = _alloc((n * 2, nbr, 4 * H), torch.float32, dev)
    recs = (GruBwdRec * (2 * n))()
    for ti in range(n):
        for d in range(2):
            r = recs[ti * 2 + d]
            r.save = S[ti][d].data_ptr()
            r.y = Y[ti][:, d * H:].data_ptr()
            r.dy = dY[ti][:, d * H:].data_ptr() if dY is not None else None
            r.dfinal = dfinal[ti][:, d * H:].data_ptr() if dfinal is not None else None
            r.whh = packs[ti].whh[layer][d].data_ptr()
            r.dgx = dG[ti][:, d * 3 * H:].data_ptr()
            r.dgh = dG[ti][:, 6 * H + d * H:].data_ptr()
            r.dhstate = dhs[ti * 2 + d].data_ptr()
            r.dbias_part = part[ti * 2 + d].data_ptr()
            r.dir = d
    ldf = dfinal[0].shape[1] if dfinal is not None else 0
    # algorithmic bytes per (row, unit): saved 4 + h_{s-1} 1 (+ dY 1) + dgh_{s+1} 3 (GEMM
    # operand) + 4 written gradients (r, z, n, W_hn h) + the carry read and written (unless
    # the kernel keeps it on chip), all of dt
    esz = 2 if dt == torch.bfloat16 else 4
    nl = lib.tt_gru_bwd_launches(dtype_code(dt), T, H)
    carry = 0 if lib.tt_gru_bwd_carry_on_chip(dtype_code(dt), T, H) else 2
    per = esz * (12 + carry + (1 if dY is not None else 0))
    kname = (f"gru_bwd_rows<{H}>" if nl == 1 else
             "gru_bwd_big" if dt == torch.bfloat16 and H % 256 == 0 and _lib.get_option("gru_bwd_big") else "gru_bwd_step<")
    with timing.region("gru_bwd", nl, 2.0 * B * 3 * H * H * 2 * n * (T - 1), float(B * T * H * 2 * n * per),
                       kernel=kname):
        call("tt_gru_bwd", dtype_code(dt), recs, 2 * n, B, T, H, 2 * H, 8 * H, ldf, stream_ptr(dev))
    sums = _alloc((n * 2, 4 * H), torch.float32, dev)
    for i in range(2 * n):
        ops.colsum(part[i], nbr, 4 * H, 4 * H, sums[i])
    dbih = [[sums[ti * 2 + d, : 3 * H] for d in range(2)] for ti in range(n)]
    dbhh = [[torch.cat([sums[ti * 2 + d, : 2 * H], sums[ti * 2 + d, 3 * H:]]) for d in range(2)] for ti in range(n)]
    return dG, dbih, dbhh


_WGRAD_T = os.environ.get("TT_WGRAD_T", "1") != "0"  # layer-0 dW_ih as its transpose (read once)
# layer-1 weight gradients on a second stream, beside the layer-0 BPTT (see TowersFn.backward).
# Off: measured slower -- sharing the CUs stretched the layer-0 BPTT from 5.9 to ~14 ms, so
# 154.4-154.8k became 152.3-152.5k pairs/s (profiles/r06_wgrad_overlap_ab.txt)
WGRAD_OVERLAP = os.environ.get("TT_WGRAD_OVERLAP", "0") == "1"
_wgrad_streams: dict = {}


def _wgrad_stream(dev) -> torch.cuda.Stream:
    dev = torch.device(dev)
    with _status_lock:
        s = _wgrad_streams.get(dev)
        if s is None:
            s = _wgrad_streams[dev] = torch.cuda.Stream(device=dev)
    return s


def _weight_grads(cfg, B, T, dG, Xin, K, ldx, Y, kr=None):
    """dW_ih = dG^T Xin, dW_hh = dGH^T Y_{t-1} for all (tower, dir) in two batched TN GEMMs."""
    n, H, dt, dev = cfg.ntowers, cfg.H, cfg.dtype, dG[0].device
    BT = B * T
    dWih = [[_alloc((3 * H, K), torch.float32, dev) for _ in range(2)] for _ in range(n)]
    dWhh = [[_alloc((3 * H, H), torch.float32, dev) for _ in range(2)] for _ in range(n)]
    a_ih, b_ih, c_ih, a_hh, a_hi, b_hh, c_hh, sh = [], [], [], [], [], [], [], []
    for ti in range(n):
        for d in range(2):
            a_ih.append(dG[ti][:, d * 3 * H:])
            b_ih.append(Xin[ti])
            c_ih.append(dWih[ti][d])
            a_hh.append(dG[ti][:, d * 3 * H:])
            a_hi.append(dG[ti][:, 6 * H + d * H:])
            b_hh.append(Y[ti][:, d * H:])
            c_hh.append(dWhh[ti][d])
            sh.append(-1 if d == 0 else 1)
    esz = 2 if dt == torch.bfloat16 else 4
    kr = K if kr is None else kr  # layer 0: the real embedding columns, not the padding
    with timing.region("wgrad_ih", 1, 2.0 * 3 * H * kr * BT * 2 * n,
                       float(n * (esz * BT * (6 * H + kr) + 2 * 3 * H * kr * 4))):
        if _WGRAD_T and dt == torch.bfloat16 and 0 < K % 256 <= 128:
            # layer 0 (K = Ep 320): dW_ih^T = Xin^T dG puts the padded width on M, where the
            # tail tile's second wave row lies wholly past M and skips its MFMAs (the
            # 256x256 loop, tt_gemm_core.h Loop8::quad): 1.5 tiles of work per 256 gate
            # rows instead of 2 for the N tail
            cT = [_alloc((K, 3 * H), torch.float32, dev) for _ in c_ih]
            ops.gemm(b_ih, a_ih, cT, m=K, n=3 * H, k=BT, lda=ldx, ldb=8 * H, ldc=3 * H, a_kouter=True,
                     b_kouter=True, dtype=dt, out_dtype=torch.float32)
            for c, ct in zip(c_ih, cT):
                c.copy_(ct.t())
        else:
            ops.gemm(a_ih, b_ih, c_ih, m=3 * H, n=K, k=BT, lda=8 * H, ldb=ldx, ldc=K, a_kouter=True,
                     b_kouter=True, dtype=dt, out_dtype=torch.float32)
    with timing.region("wgrad_hh", 1, 2.0 * 3 * H * H * BT * 2 * n,
                       float(n * (esz * BT * (6 * H + 2 * H) + 2 * 3 * H * H * 4))):
        ops.gemm(a_hh, b_hh, c_hh, m=3 * H, n=H, k=BT, lda=8 * H, ldb=2 * H, ldc=H, a_kouter=True, b_kouter=True,
                 dtype=dt, out_dtype=torch.float32, bshift=sh, seq_t=T, a_hi=a_hi, a_split=2 * H)
    return dWih, dWhh


class TowersFn(torch.autograd.Function):
    """(x_0..x_{n-1}, params...) -> (vec_0..vec_{n-1}), vec_i = tower_i(x_i) as [B, h] fp32
    (cfg.head "proj2"), or the final bidirectional state cat(h_fwd, h_rev) as [B, 2H] fp32
    (cfg.head "none": margin_two_tower.py:59-61, the head runs outside)."""

    @staticmethod
    def forward(ctx, cfg: TowerCfg, table, group, cache_ok, *args):
        n = cfg.ntowers
        xs, params = args[:n], args[n:]
        _lib.require_gpu(*xs, *params)
        check_gru_status(wait=True)  # every earlier forward's column-split launches
        dt, E, H, h = cfg.dtype, cfg.E, cfg.H, cfg.h
        dev = xs[0].device
        reset_guard_if_reported(dev)
        B, T = xs[0].shape[0], xs[0].shape[1]
        for x in xs:
            if x.shape[0] != B or x.shape[1] != T:
                raise ValueError("query and doc inputs must share [B, T] in one fused call")
        Ep = ops.pad_cols(E, dt)
        npt = cfg.nparams
        packs = [_packed(params[i * npt:(i + 1) * npt], cfg, Ep, cache_ok) for i in range(n)]
        X0 = [featurize(x, table, Ep, dt) for x in xs]
        train_drop = cfg.drop_p > 0.0
        seeds = [int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) for _ in range(n)] if train_drop else [0] * n
        # one workspace for both layers (same shape; the launches are stream-ordered)
        ws = gru_fwd_workspace(2 * n, B, T, H, dt, dev)
        Y0, X1, S0 = _gru_layer_fwd(cfg, X0, Ep, Ep, packs, 0, B, T, seeds, train_drop, ws)
        Xl1 = X1 if train_drop else Y0
        Y1, _, S1 = _gru_layer_fwd(cfg, Xl1, 2 * H, 2 * H, packs, 1, B, T, seeds, False, ws)
        if ws is not None:
            # only a forward that records autograd state arms the optimiser's step guard
            watch_gru_status(ws, arm=any(ctx.needs_input_grad))
        # cat(h_fwd at t=T-1, h_rev at t=0) -> [B, 2H] (enhanced_two_tower.py:53,59)
        hcat = []
        for ti in range(n):
            y = Y1[ti].view(B, T, 2 * H)
            hcat.append(torch.cat([y[:, T - 1, :H], y[:, 0, H:]], 1).to(HEAD_DT).contiguous())
        ctx.cfg = cfg
        ctx.group = group
        ctx.params = params
        ctx.dims = (B, T, Ep)
        ctx.seeds = seeds
        ctx.packs = packs
        if cfg.head == "none":
            ctx.acts = (X0, Y0, X1, S0, Y1, S1, None, None, None, None, None)
            return tuple(hcat)
        outs, p1s, means, rstds, us = [], [], [], [], []
        io = (HeadFwdIO * n)()
        for ti in range(n):
            pk = packs[ti]
            p1 = _alloc((B, 2 * h), HEAD_DT, dev)
            u = _alloc((B, 2 * h), HEAD_DT, dev)
            mean = _alloc((B,), torch.float32, dev)
            rstd = _alloc((B,), torch.float32, dev)
            out = _alloc((B, h), torch.float32, dev)
            q = io[ti]
            q.w1, q.b1, q.ln_g, q.ln_b = pk.w1.data_ptr(), pk.b1.data_ptr(), pk.ln_g.data_ptr(), pk.ln_b.data_ptr()
            q.w2, q.b2 = pk.w2.data_ptr(), pk.b2.data_ptr()
            q.x, q.p1, q.mean, q.rstd, q.u, q.out = (hcat[ti].data_ptr(), p1.data_ptr(), mean.data_ptr(),
                                                     rstd.data_ptr(), u.data_ptr(), out.data_ptr())
            outs.append(out); p1s.append(p1); means.append(mean); rstds.append(rstd); us.append(u)
        call("tt_proj_head_fwd", dtype_code(HEAD_DT), io, n, B, h, LN_EPS, stream_ptr(dev))
        ctx.acts = (X0, Y0, X1, S0, Y1, S1, hcat, p1s, means, rstds, us)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        cfg = ctx.cfg
        check_gru_status(wait=False)  # the forwards that have finished by now
        n, dt, E, H, h = cfg.ntowers, cfg.dtype, cfg.E, cfg.H, cfg.h
        B, T, Ep = ctx.dims
        packs = ctx.packs
        X0, Y0, X1, S0, Y1, S1, hcat, p1s, means, rstds, us = ctx.acts
        dev = Y0[0].device
        lib = _lib.load()
        st = stream_ptr(dev)
        # ---- projection head
        head_grads = [[] for _ in range(n)]
        dhcat = []
        if cfg.head == "none":
            for ti in range(n):
                g = gouts[ti]
                dhcat.append(torch.zeros(B, 2 * H, dtype=torch.float32, device=dev) if g is None
                             else g.float().contiguous())
        ws = None
        if cfg.head == "proj2":
            ws = _alloc((lib.tt_proj_head_bwd_ws_size(dtype_code(HEAD_DT), B, h),), torch.uint8, dev)
        for ti in range(n if cfg.head == "proj2" else 0):
            g = gouts[ti]
            g = torch.zeros(B, h, dtype=torch.float32, device=dev) if g is None else g.float().contiguous()
            pk = packs[ti]
            dx = _alloc((B, 2 * H), torch.float32, dev)
            dw1 = _alloc(pk.w1.shape, torch.float32, dev)
            db1 = _alloc((2 * h,), torch.float32, dev)
            dg = _alloc((2 * h,), torch.float32, dev)
            dbeta = _alloc((2 * h,), torch.float32, dev)
            dw2 = _alloc(pk.w2.shape, torch.float32, dev)
            db2 = _alloc((h,), torch.float32, dev)
            io = HeadBwdIO()
            io.w1, io.ln_g, io.ln_b, io.w2 = pk.w1.data_ptr(), pk.ln_g.data_ptr(), pk.ln_b.data_ptr(), pk.w2.data_ptr()
            io.x, io.p1, io.mean, io.rstd, io.u = (hcat[ti].data_ptr(), p1s[ti].data_ptr(), means[ti].data_ptr(),
                                                   rstds[ti].data_ptr(), us[ti].data_ptr())
            io.dout, io.dx = g.data_ptr(), dx.data_ptr()
            io.dw1, io.db1, io.dg, io.dbeta, io.dw2, io.db2 = (dw1.data_ptr(), db1.data_ptr(), dg.data_ptr(),
                                                               dbeta.data_ptr(), dw2.data_ptr(), db2.data_ptr())
            io.ws = ws.data_ptr()
            call("tt_proj_head_bwd", dtype_code(HEAD_DT), ctypes.byref(io), 1, B, h, LN_EPS, st)
            head_grads[ti] = [dw1, db1, dg, dbeta, dw2, db2]
            dhcat.append(dx)
        # ---- GRU layer 1: dfinal enters at the last processed step of each direction
        dG1, dbih1, dbhh1 = _gru_layer_bwd(cfg, 1, B, T, S1, Y1, None, dhcat, packs)
        Xl1 = X1 if X1 is not None else Y0
        red = dist.OverlapReducer(ctx.group[0]) if ctx.group is not None else None
        gl = [{} for _ in range(n)]

        def layer1_wgrads():
            dWih1, dWhh1 = _weight_grads(cfg, B, T, dG1, Xl1, 2 * H, 2 * H, Y1)
            _layer_grads(gl, 1, E, Ep, dWih1, dWhh1, dbih1, dbhh1)
            # data-parallel: the head + layer-1 gradients are summed across ranks while the
            # layer-0 BPTT below runs (dist.OverlapReducer)
            if red is not None:
                _reduce_into(red, gl, head_grads)

        # The layer-1 weight gradients (MFMA-bound TN GEMMs) do not feed the layer-0 BPTT
        # (HBM-bound, row-owning: no co-residency requirement), so with WGRAD_OVERLAP they run on
        # a second stream beside it; the layer-1 data gradient, which the BPTT needs, goes first.
        main = torch.cuda.current_stream(dev)
        side = _wgrad_stream(dev) if WGRAD_OVERLAP else None
        if side is None:
            layer1_wgrads()
        # dL/dY0 = (dG1 Wih1) * dropout mask  [B*T, 2H]
        dY0 = [_alloc((B * T, 2 * H), dt, dev) for _ in range(n)]
        esz = 2 if dt == torch.bfloat16 else 4
        with timing.region("dgrad_l1", 1, 2.0 * B * T * 2 * H * 6 * H * n,
                           float(n * esz * (B * T * 6 * H + B * T * 2 * H))):
            if X1 is None:
                ops.gemm(dG1, [p.wih[1] for p in packs], dY0, m=B * T, n=2 * H, k=6 * H, lda=8 * H, ldb=2 * H,
                         ldc=2 * H, a_kouter=False, b_kouter=True, dtype=dt, out_dtype=dt)
            else:
                for ti in range(n):
                    ops.gemm([dG1[ti]], [packs[ti].wih[1]], [dY0[ti]], m=B * T, n=2 * H, k=6 * H, lda=8 * H,
                             ldb=2 * H, ldc=2 * H, a_kouter=False, b_kouter=True, dtype=dt, out_dtype=dt,
                             drop_seed=ctx.seeds[ti], drop_p=cfg.drop_p, drop_row0=cfg.rank * B * T)
        if side is not None:
            side.wait_stream(main)
            for t in (*dG1, *Xl1, *Y1, *[g for hg in head_grads for g in hg], *[x for b in dbih1 for x in b],
                      *[x for b in dbhh1 for x in b]):
                t.record_stream(side)  # read on the side stream after main drops them
            with torch.cuda.stream(side):
                layer1_wgrads()
        del dG1
        # ---- GRU layer 0
        dG0, dbih0, dbhh0 = _gru_layer_bwd(cfg, 0, B, T, S0, Y0, dY0, None, packs)
        del dY0
        dWih0, dWhh0 = _weight_grads(cfg, B, T, dG0, X0, Ep, Ep, Y0, kr=E)
        gl0 = [{} for _ in range(n)]
        _layer_grads(gl0, 0, E, Ep, dWih0, dWhh0, dbih0, dbhh0)
        if side is not None:
            main.wait_stream(side)
            for t in [*[v for d in gl for v in d.values()], *[g for hg in head_grads for g in hg]]:
                t.record_stream(main)  # made on the side stream, used (and freed) on main
        if red is not None:
            _reduce_into(red, gl0, [[] for _ in range(n)])
            red.finish(ctx.params)
        grads = []
        for ti in range(n):
            gl[ti].update(gl0[ti])
            grads.extend(gl[ti][k] for k in GRU_NAMES)
            grads.extend(head_grads[ti])
        ctx.acts = None
        ctx.packs = None
        ctx.params = None
        return (None, None, None, None, *([None] * n), *grads)


def _layer_grads(gl, layer, E, Ep, dWih, dWhh, dbih, dbhh):
    """Per-tower {name: grad} of one GRU layer in the nn.GRU parameter layout."""
    for ti in range(len(gl)):
        for d, sfx in enumerate(("", "_reverse")):
            w = dWih[ti][d]
            if layer == 0 and Ep != E:
                w = w[:, :E].contiguous()
            gl[ti][f"weight_ih_l{layer}{sfx}"] = w
            gl[ti][f"weight_hh_l{layer}{sfx}"] = dWhh[ti][d]
            gl[ti][f"bias_ih_l{layer}{sfx}"] = dbih[ti][d].contiguous()
            gl[ti][f"bias_hh_l{layer}{sfx}"] = dbhh[ti][d]


def _reduce_into(red, gl, head_grads):
    """Start one bucket's all-reduce and swap the gradients for views of the bucket."""
    keys = [(ti, k) for ti in range(len(gl)) for k in gl[ti]]
    heads = [(ti, j) for ti in range(len(head_grads)) for j in range(len(head_grads[ti]))]
    views = red.launch([gl[ti][k] for ti, k in keys] + [head_grads[ti][j] for ti, j in heads])
    for (ti, k), v in zip(keys, views):
        gl[ti][k] = v
    for (ti, j), v in zip(heads, views[len(keys):]):
        head_grads[ti][j] = v


def run_towers(cfg: TowerCfg, table, xs, params, reduce_group=None, reduce: bool = False):
    """reduce: sum the gradients across the data-parallel reduce_group's ranks during the
    backward (dist.OverlapReducer); ignored unless that group spans more than one rank."""
    if cfg.H % 8:
        raise ValueError(f"GRU hidden size {cfg.H} must be a multiple of 8 on the HIP path "
                         "(the step epilogues update 8 consecutive units per thread)")
    group = (reduce_group,) if reduce and dist.active(reduce_group) else None
    # inference (no gradient wanted): the packed compute copies may be reused while the
    # parameters are unchanged (retrieval / serving encode many batches per weight version)
    cache_ok = not (torch.is_grad_enabled() and any(p.requires_grad for p in params))
    return TowersFn.apply(cfg, table, group, cache_ok, *xs, *params)
