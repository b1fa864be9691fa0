"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL ("nccl").

The reference has no parallelism. The DP step here:
  forward : all-gather the normalised doc vectors so every rank scores its queries
            against the global negative pool (labels offset by rank * B_local);
  backward: reduce-scatter (sum) the gradient wrt the gathered doc vectors back to the
            rank that owns each row; all-reduce (sum) the parameter gradients.
Each rank's loss is its rows' share of the GLOBAL mean (divided by the global batch),
so the summed gradients are exactly the single-process gradients of the whole batch.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def forced() -> bool:
    """TT_DIST_FORCE=1: run every collective even in a one-rank process group, so the DP
    path's RCCL calls (all-gather, reduce-scatter, bucketed and overlapped all-reduce)
    execute on a single GPU (tests/test_gpu_dist.py, bench.py rehearsal)."""
    return os.environ.get("TT_DIST_FORCE", "0") == "1"


def active(group=None) -> bool:
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size(group) > 1 or forced()


def rank_world(group=None):
    if not active(group):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def all_gather_rows(x: torch.Tensor, group=None) -> torch.Tensor:
    """[B_l, ...] on every rank -> [world * B_l, ...] in rank order (no autograd)."""
    if not active(group):
        return x
    r, w = rank_world(group)
    out = torch.empty((w * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x.contiguous(), group=group)
    return out


def reduce_scatter_rows(x: torch.Tensor, group=None) -> torch.Tensor:
    """[world * B_l, ...] partial sums on every rank -> this rank's [B_l, ...] total."""
    if not active(group):
        return x
    r, w = rank_world(group)
    out = torch.empty((x.shape[0] // w,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x.contiguous(), op=dist.ReduceOp.SUM, group=group)
    return out


def all_reduce_sum_(t: torch.Tensor, group=None):
    if active(group):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


class GatherRows(torch.autograd.Function):
    """Differentiable all-gather: backward reduce-scatters the gradient."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return all_gather_rows(x, group)

    @staticmethod
    def backward(ctx, g):
        return reduce_scatter_rows(g, ctx.group), None


class OverlapReducer:
    """Gradient buckets summed across ranks while the backward keeps running.

    TowersFn.backward hands over the head + layer-1 gradients as soon as they exist
    (launch) and runs the layer-0 BPTT while that all-reduce is on the wire; the layer-0
    bucket follows, then finish() waits for both. Each bucket is one flat fp32
    collective (RCCL: on its own stream, ordered after the kernels that produced the
    bucket); the returned views of the reduced buffer become the parameters' gradients,
    and the parameters are marked so allreduce_grads does not sum them a second time."""

    def __init__(self, group=None):
        self.group = group
        self.works = []

    def launch(self, grads):
        flat = torch.cat([g.reshape(-1).float() for g in grads])
        self.works.append(dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        out, off = [], 0
        for g in grads:
            out.append(flat[off:off + g.numel()].view(g.shape))
            off += g.numel()
        return out

    def finish(self, params=()):
        for w in self.works:
            w.wait()
        self.works = []
        for p in params:
            p._tt_dp_reduced = True


def allreduce_grads(params, group=None, bucket_bytes: int = 64 << 20):
    """Sum parameter gradients across ranks in flat buckets (one collective per
    ~64 MB bucket: xGMI rings are per-link bound, so few large collectives win).
    Gradients an OverlapReducer already summed during the backward are skipped."""
    if not active(group):
        return
    grads = []
    for p in params:
        if getattr(p, "_tt_dp_reduced", False):
            p._tt_dp_reduced = False
        elif p.grad is not None:
            grads.append(p.grad)
    bucket, size = [], 0
    for g in grads + [None]:
        if g is not None:
            bucket.append(g)
            size += g.numel() * g.element_size()
        if bucket and (g is None or size >= bucket_bytes):
            flat = torch.cat([b.reshape(-1) for b in bucket])
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
            off = 0
            for b in bucket:
                b.copy_(flat[off:off + b.numel()].view_as(b))
                off += b.numel()
            bucket, size = [], 0
