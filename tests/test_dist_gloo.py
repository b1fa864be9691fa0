"""Data-parallel host logic (two_towers_amd/dist.py) at world_size 2 over gloo on CPU.

The loss math here is the oracle's (CPU); what is under test is the DP plumbing the
GPU path uses unchanged: GatherRows (all-gather forward / reduce-scatter backward),
the global-mean loss split, and the bucketed gradient all-reduce. Two ranks holding
half a batch each must reproduce the single-process gradients of the whole batch."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from oracle import cpu_ref


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_loss(p, q, d, group, rank, world):
    from two_towers_amd import dist as tdp
    qv, dv = cpu_ref.forward(q, d, p)
    qn, dn = cpu_ref.normalize(qv), cpu_ref.normalize(dv)
    dn_all = tdp.GatherRows.apply(dn.contiguous(), group)
    B = q.shape[0]
    s = qn @ dn_all.t() / 0.07
    labels = torch.arange(B) + rank * B
    local_sum = torch.nn.functional.cross_entropy(s, labels, reduction="sum")
    loss = local_sum / (B * world)
    tot = loss.detach().clone()
    tdp.all_reduce_sum_(tot, group)
    return loss + (tot - loss.detach())


def _worker(rank, world, port, q, d, p0, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from two_towers_amd import dist as tdp
    B = q.shape[0] // world
    p = {k: v.clone().requires_grad_(True) for k, v in p0.items()}
    loss = _dp_loss(p, q[rank * B:(rank + 1) * B], d[rank * B:(rank + 1) * B], None, rank, world)
    loss.backward()
    params = list(p.values())
    for t in params:
        t.grad = t.grad.contiguous()
    tdp.allreduce_grads(params, None, bucket_bytes=4096)
    if rank == 0:
        out.put((float(loss.detach()), {k: v.grad.numpy().copy() for k, v in p.items()}))  # by value
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_dp_gather_loss_and_grads_match_single_process(world):
    torch.manual_seed(0)
    p0 = cpu_ref.counter_params(12, 8, 3)
    g = torch.Generator().manual_seed(4)
    q = torch.randn(16, 5, 12, generator=g)
    d = torch.randn(16, 5, 12, generator=g)
    ref_p = {k: v.clone().requires_grad_(True) for k, v in p0.items()}
    ref_loss = cpu_ref.infonce(*cpu_ref.forward(q, d, ref_p))
    ref_loss.backward()
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, d, p0, out)) for r in range(world)]
    for pr in procs:
        pr.start()
    loss, grads = out.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert abs(loss - float(ref_loss)) < 1e-5
    for k, v in ref_p.items():
        torch.testing.assert_close(torch.from_numpy(grads[k]), v.grad, rtol=1e-4, atol=1e-6)


def _overlap_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from two_towers_amd import dist as tdp
        g = torch.Generator().manual_seed(10 + rank)
        # two buckets in flight at once, as TowersFn.backward launches them (head + layer
        # 1, then layer 0), then the skip logic of allreduce_grads
        a = [torch.randn(3, 5, generator=g), torch.randn(7, generator=g)]
        b = [torch.randn(4, 2, generator=g)]
        red = tdp.OverlapReducer(None)
        va = red.launch(a)
        vb = red.launch(b)
        params = [torch.nn.Parameter(torch.zeros(3, 5)), torch.nn.Parameter(torch.zeros(2))]
        params[1].grad = torch.full((2,), float(rank + 1))
        red.finish(params[:1])
        params[0].grad = va[0]
        tdp.allreduce_grads(params, None)  # sums params[1] only
        out.put((rank, [v.numpy().copy() for v in va + vb], params[0].grad.numpy().copy(),
                 params[1].grad.numpy().copy(), params[0]._tt_dp_reduced, [x.numpy().copy() for x in a + b]))
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


def test_overlap_reducer_buckets_and_skip():
    """dist.OverlapReducer (the backward's in-flight gradient buckets): two async buckets
    at world 2 sum to the per-rank totals with their shapes kept; allreduce_grads skips
    (and unmarks) the parameters the reducer already summed and still sums the rest."""
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, out)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict((r[0], r[1:]) for r in (out.get(timeout=120), out.get(timeout=120)))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    srcs = [res[r][4] for r in range(2)]
    for r in range(2):
        views, g0, g1, flag, _ = res[r]
        for i, v in enumerate(views):
            assert v.shape == srcs[0][i].shape
            torch.testing.assert_close(torch.from_numpy(v), torch.from_numpy(srcs[0][i] + srcs[1][i]))
        torch.testing.assert_close(torch.from_numpy(g0), torch.from_numpy(srcs[0][0] + srcs[1][0]))
        assert (g1 == 3.0).all()  # 1 + 2: summed once by allreduce_grads
        assert flag is False
