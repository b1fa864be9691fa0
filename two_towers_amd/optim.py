"""Adam for the inner loop of train_enhanced.py:43,63 as one multi-tensor HIP launch.

Same hyper-parameters and update formula as torch.optim.Adam (non-amsgrad,
non-maximize); state lives in fp32 tensors per parameter ('exp_avg', 'exp_avg_sq',
'step' like torch, so optimizer.state_dict() keeps torch's structure).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, towers
from ._lib import call, stream_ptr

_MAXT = 48


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0.0 or eps < 0.0 or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError("invalid Adam hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._guard_reads = []  # (event, pinned int32[1] copy of the guard, params) per earlier launch

    def settle_skipped_steps(self):
        """Take every earlier step that the device skipped (its step guard was set) off the
        step counters of the parameters it covered, so Adam's bias correction counts applied
        updates only. Called by step(); waits for the earlier steps' launches (the host is
        normally a whole forward and backward ahead of them, so this rarely blocks)."""
        reads, self._guard_reads = self._guard_reads, []
        for ev, word, plist in reads:
            ev.synchronize()
            if int(word.item()) != 0:
                for p in plist:
                    self.state[p]["step"] -= 1

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.settle_skipped_steps()
        stepped = {}  # device -> parameters launched this step
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            _lib.require_gpu(*ps)
            b1, b2 = group["betas"]
            # torch keeps one step counter per parameter; parameters stepped together share it
            buckets = {}
            for p in ps:
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if p.dtype != torch.float32 or not p.is_contiguous() or not p.grad.is_contiguous():
                    raise _lib.TTError("two_towers_amd Adam expects contiguous fp32 parameters and gradients")
                st["step"] += 1
                buckets.setdefault(int(st["step"].item()), []).append(p)
            # the device's step guard: non-zero when a column-split GRU forward since the
            # last step timed out (towers.watch_gru_status); the kernel then changes nothing
            dev = ps[0].device
            guard = towers.step_guard(dev)
            for step, plist in buckets.items():
                for i in range(0, len(plist), _MAXT):
                    chunk = plist[i:i + _MAXT]
                    n = len(chunk)
                    arr = lambda xs: (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])
                    sizes = (ctypes.c_long * n)(*[p.numel() for p in chunk])
                    call("tt_adam_multi", arr(chunk), arr([p.grad for p in chunk]),
                         arr([self.state[p]["exp_avg"] for p in chunk]),
                         arr([self.state[p]["exp_avg_sq"] for p in chunk]), sizes, n, group["lr"], b1, b2,
                         group["eps"], group["weight_decay"], step, guard.data_ptr(), stream_ptr(dev))
            # the kernel writes through raw pointers: record the in-place update for autograd
            # and for the packed-weight cache of the towers (towers._packed)
            torch.autograd.graph.increment_version(ps)
            stepped.setdefault(dev, []).extend(ps)
        for dev, plist in stepped.items():
            g = towers.step_guard(dev)
            with torch.cuda.device(dev):
                word = torch.zeros(1, dtype=torch.int32, pin_memory=True)
                word.copy_(g, non_blocking=True)  # did the device skip this step? (settle_skipped_steps)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(dev))
                g.zero_()  # stream-ordered after every launch above
            self._guard_reads.append((ev, word, plist))
        return loss
