"""Contrastive losses of enhanced_two_tower.py on the HIP path.

  InfoNCELoss(temperature=0.07)                 enhanced_two_tower.py:67-82
  MarginRankingLoss(margin=0.2, temperature=0.1) enhanced_two_tower.py:84-121
  get_hard_negatives(q, docs, positive_idx, k)   enhanced_two_tower.py:123-133
  HardNegativeMarginLoss(k=5, margin=0.2)        the config-3 composition:
      mine k hard negatives per query among the (global) doc pool, then the
      explicit-negative MarginRankingLoss — fused, without gathering negative rows.

Every loss takes an optional torch.distributed process group: with world > 1 the
normalised doc vectors are all-gathered (global negative pool) and each rank returns
the GLOBAL mean loss while back-propagating only its own rows' share (see dist.py).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib, dist, ops, timing
from ._lib import call, dtype_code, ptr, stream_ptr


def _dt_of(x: torch.Tensor, compute_dtype):
    return compute_dtype if compute_dtype is not None else torch.float32


def _finish_loss(local_sum: torch.Tensor, scale: float, group):
    """local_sum * scale as this rank's differentiable share; value = global mean."""
    loss = local_sum * scale
    if dist.active(group):
        tot = loss.detach().clone()
        dist.all_reduce_sum_(tot, group)
        loss = loss + (tot - loss.detach())
    return loss


class _NormCE(torch.autograd.Function):
    """sum_i CE_i over S = inv_tau * qn dn_global^T (- offdiag off the label), with
    qn/dn = normalize(q/d) (or raw when normalize=False). Returns the local row sum."""

    @staticmethod
    def forward(ctx, q, d, inv_tau, offdiag, eps, do_norm, dt, group):
        _lib.require_gpu(q, d)
        q = q.float().contiguous()
        d = d.float().contiguous()
        rank, world = dist.rank_world(group)
        B = q.shape[0]
        if do_norm:
            qn, qn32, qnorm = ops.l2norm_fwd(q, eps, dt)
            dn_l, dn32, dnorm = ops.l2norm_fwd(d, eps, dt)
        else:
            qn, qn32, qnorm = (q if dt == torch.float32 else q.to(dt)), q, None
            dn_l, dn32, dnorm = (d if dt == torch.float32 else d.to(dt)), d, None
        dn = dist.all_gather_rows(dn_l, group)
        nd = dn.shape[0]
        lse = torch.empty(B, dtype=torch.float32, device=q.device)
        row = torch.empty(B, dtype=torch.float32, device=q.device)
        lib = _lib.load()
        ws = torch.empty(lib.tt_infonce_fwd_ws_size(B, nd), dtype=torch.uint8, device=q.device)
        esz = 2 if dt == torch.bfloat16 else 4
        with timing.region("infonce_fwd", 1, 2.0 * B * nd * q.shape[1], float(esz * (B + nd) * q.shape[1] + 8 * B)):
            call("tt_infonce_fwd", dtype_code(dt), qn.data_ptr(), B, dn.data_ptr(), nd, q.shape[1], inv_tau,
                 offdiag, rank * B, lse.data_ptr(), row.data_ptr(), ws.data_ptr(), stream_ptr(q.device))
        out = torch.empty((), dtype=torch.float32, device=q.device)
        ops.total(row, 1.0, out)
        ctx.save = (qn, qn32, qnorm, dn, dn32, dnorm, lse)
        ctx.cfg = (inv_tau, offdiag, eps, do_norm, dt, group, rank, B)
        return out

    @staticmethod
    def backward(ctx, gout):
        qn, qn32, qnorm, dn, dn32, dnorm, lse = ctx.save
        inv_tau, offdiag, eps, do_norm, dt, group, rank, B = ctx.cfg
        h = qn.shape[1]
        nd = dn.shape[0]
        # the scalar upstream gradient stays on the device: the kernels read it
        gdev = gout.detach().float().reshape(1).contiguous()
        dqn = torch.empty(B, h, dtype=torch.float32, device=qn.device)
        ddn = torch.empty(nd, h, dtype=torch.float32, device=qn.device)
        lib = _lib.load()
        ws = torch.empty(lib.tt_infonce_bwd_ws_size(dtype_code(dt), B, nd, h), dtype=torch.uint8, device=qn.device)
        call("tt_infonce_bwd", dtype_code(dt), qn.data_ptr(), B, dn.data_ptr(), nd, h, inv_tau, offdiag, rank * B,
             lse.data_ptr(), gdev.data_ptr(), dqn.data_ptr(), ddn.data_ptr(), ws.data_ptr(), stream_ptr(qn.device))
        ddn_l = dist.reduce_scatter_rows(ddn, group)
        if do_norm:
            dq = ops.l2norm_bwd(dqn, qn32, qnorm, eps)
            dd = ops.l2norm_bwd(ddn_l, dn32, dnorm, eps)
        else:
            dq, dd = dqn, ddn_l
        return dq, dd, None, None, None, None, None, None


class InfoNCELoss(nn.Module):
    """enhanced_two_tower.py:67-82: CE over normalised q·dᵀ / temperature, labels = arange."""

    def __init__(self, temperature=0.07, compute_dtype=None, process_group=None):
        super().__init__()
        self.temperature = temperature
        self.compute_dtype = compute_dtype
        self.process_group = process_group

    def forward(self, query_vec, doc_vec):
        dt = _dt_of(query_vec, self.compute_dtype)
        _, world = dist.rank_world(self.process_group)
        s = _NormCE.apply(query_vec, doc_vec, 1.0 / self.temperature, 0.0, 1e-12, True, dt, self.process_group)
        return _finish_loss(s, 1.0 / (query_vec.shape[0] * world), self.process_group)


class _MarginFn(torch.autograd.Function):
    """sum_i relu(margin - cos(q_i, dpool[lab_i]) + mean_j cos(q_i, dpool[idx_ij]))."""

    @staticmethod
    def forward(ctx, q, dpool, idx, label_offset, margin, eps):
        _lib.require_gpu(q, dpool)
        q = q.float().contiguous()
        dpool = dpool.float().contiguous()
        qn, _, qnorm = ops.l2norm_fwd(q, eps, torch.float32)
        dn, _, dnorm = ops.l2norm_fwd(dpool, eps, torch.float32)
        B, h = q.shape
        k = idx.shape[1]
        row = torch.empty(B, dtype=torch.float32, device=q.device)
        call("tt_margin_fwd", qn.data_ptr(), B, dn.data_ptr(), dn.shape[0], h, label_offset, idx.data_ptr(), k,
             margin, row.data_ptr(), stream_ptr(q.device))
        out = torch.empty((), dtype=torch.float32, device=q.device)
        ops.total(row, 1.0, out)
        ctx.save = (qn, qnorm, dn, dnorm, idx)
        ctx.cfg = (label_offset, margin, eps)
        return out

    @staticmethod
    def backward(ctx, gout):
        qn, qnorm, dn, dnorm, idx = ctx.save
        label_offset, margin, eps = ctx.cfg
        B, h = qn.shape
        dqn = torch.empty_like(qn)
        ddn = torch.zeros_like(dn)
        ws = torch.empty(_lib.load().tt_margin_bwd_ws_size(B, dn.shape[0], h, idx.shape[1]), dtype=torch.uint8, device=qn.device)
        gdev = gout.detach().float().reshape(1).contiguous()  # read by the kernels: no host sync
        call("tt_margin_bwd", qn.data_ptr(), B, dn.data_ptr(), dn.shape[0], h, label_offset, idx.data_ptr(),
             idx.shape[1], margin, gdev.data_ptr(), dqn.data_ptr(), ddn.data_ptr(), ws.data_ptr(),
             stream_ptr(qn.device))
        return ops.l2norm_bwd(dqn, qn, qnorm, eps), ops.l2norm_bwd(ddn, dn, dnorm, eps), None, None, None, None


class MarginRankingLoss(nn.Module):
    """enhanced_two_tower.py:84-121.
    neg_doc_vec None: in-batch CE over q·dᵀ/τ (un-normalised) minus margin off the diagonal.
    neg_doc_vec [B*k, h] (query-major): mean(relu(margin - cos(q,pos) + mean_k cos(q,neg)))."""

    def __init__(self, margin=0.2, temperature=0.1, compute_dtype=None, process_group=None):
        super().__init__()
        self.margin = margin
        self.temperature = temperature
        self.compute_dtype = compute_dtype
        self.process_group = process_group

    def forward(self, query_vec, pos_doc_vec, neg_doc_vec=None):
        B = query_vec.shape[0]
        if neg_doc_vec is None:
            dt = _dt_of(query_vec, self.compute_dtype)
            _, world = dist.rank_world(self.process_group)
            s = _NormCE.apply(query_vec, pos_doc_vec, 1.0 / self.temperature, self.margin, 0.0, False, dt,
                              self.process_group)
            return _finish_loss(s, 1.0 / (B * world), self.process_group)
        k = neg_doc_vec.shape[0] // B
        pool = torch.cat([pos_doc_vec, neg_doc_vec], 0)
        idx = (B + torch.arange(B * k, device=query_vec.device, dtype=torch.int32)).view(B, k).contiguous()
        s = _MarginFn.apply(query_vec, pool, idx, 0, self.margin, 1e-8)
        return s / B


def mine_hard_negatives(query_vecs: torch.Tensor, doc_vecs: torch.Tensor, label_offset: int = 0, k: int = 5,
                        compute_dtype=torch.float32, eps: float = 1e-8, return_values: bool = False):
    """Batched get_hard_negatives: for row i the positive is doc label_offset + i (masked
    to -1; label_offset < 0 masks nothing). Returns int32 [B, k] sorted by descending
    cosine, ties towards the lower doc index."""
    _lib.require_gpu(query_vecs, doc_vecs)
    with torch.no_grad():
        qn, _, _ = ops.l2norm_fwd(query_vecs.float().contiguous(), eps, compute_dtype, want_f32=False)
        dn, _, _ = ops.l2norm_fwd(doc_vecs.float().contiguous(), eps, compute_dtype, want_f32=False)
        B, h = qn.shape
        nd = dn.shape[0]
        idx = torch.empty(B, k, dtype=torch.int32, device=qn.device)
        val = torch.empty(B, k, dtype=torch.float32, device=qn.device) if return_values else None
        lib = _lib.load()
        ws = torch.empty(lib.tt_hardneg_ws_size(dtype_code(compute_dtype), B, nd, h, k), dtype=torch.uint8,
                         device=qn.device)
        esz = 2 if compute_dtype == torch.bfloat16 else 4
        with timing.region("hardneg_topk", 1, 2.0 * B * nd * h, float(esz * (B + nd) * h + B * k * 4)):
            call("tt_hardneg_topk", dtype_code(compute_dtype), qn.data_ptr(), B, dn.data_ptr(), nd, h,
                 label_offset, k, idx.data_ptr(), ptr(val), ws.data_ptr(), stream_ptr(qn.device))
    return (idx, val) if return_values else idx


def get_hard_negatives(query_vec, doc_vecs, positive_idx, k=5):
    """enhanced_two_tower.py:123-133 (one query). Returns int64 indices [k]."""
    idx = mine_hard_negatives(query_vec.reshape(1, -1), doc_vecs, int(positive_idx), k)
    return idx[0].long()


class HardNegativeMarginLoss(nn.Module):
    """Config 3 of BASELINE.json: per query, mine k hard negatives among all (global)
    docs with the positive masked, then MarginRankingLoss(margin) with those negatives.
    Equivalent to the reference composition
        idx_i = get_hard_negatives(q_i, d, i, k); MarginRankingLoss()(q, d, d[cat idx])."""

    def __init__(self, k=5, margin=0.2, compute_dtype=None, process_group=None):
        super().__init__()
        self.k = k
        self.margin = margin
        self.compute_dtype = compute_dtype
        self.process_group = process_group
        self.last_indices = None

    def forward(self, query_vec, doc_vec):
        dt = _dt_of(query_vec, self.compute_dtype)
        rank, world = dist.rank_world(self.process_group)
        B = query_vec.shape[0]
        pool = dist.GatherRows.apply(doc_vec.float().contiguous(), self.process_group) if world > 1 else doc_vec
        idx = mine_hard_negatives(query_vec.detach(), pool.detach(), rank * B, self.k, dt)
        self.last_indices = idx
        s = _MarginFn.apply(query_vec, pool, idx, rank * B, self.margin, 1e-8)
        return _finish_loss(s, 1.0 / (B * world), self.process_group)
