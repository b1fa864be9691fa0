"""Thin tensor-level wrappers over the C ABI (one function per entry point family).

Every wrapper checks the operands it is handed (device, dtype, contiguity, size) so
shape mistakes fail in Python with a clear message before any kernel launches.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import torch

from . import _lib
from ._lib import GemmBatch, call, dtype_code, ptr, stream_ptr


def _esz(dt: torch.dtype) -> int:
    return 2 if dt == torch.bfloat16 else 4


def pad_cols(e: int, dt: torch.dtype) -> int:
    """Padded width of gathered embedding rows: whole 128-byte lines (one GEMM K-tile), so
    every K-tile of the layer-0 GEMMs starts on a cache line (E 300 bf16 -> 320: input
    projection l0 3.70-3.78 vs 3.82-3.85 ms per step at 304 columns, the step 0.1-1.1 %
    faster, profiles/r02_ep_align_ab.txt; the extra columns are zeros in the table and in
    W_ih l0 and add no K-tile)."""
    epc = 128 // _esz(dt)
    return (e + epc - 1) // epc * epc


def gemm(a: Sequence[torch.Tensor], b: Sequence[torch.Tensor], c: Sequence[torch.Tensor], *, m: int, n: int,
         k: int, lda: int, ldb: int, ldc: int, a_kouter: bool, b_kouter: bool, dtype: torch.dtype,
         out_dtype: torch.dtype, bias: Sequence[torch.Tensor | None] | None = None,
         bshift: Sequence[int] | None = None, alpha: float = 1.0, accumulate: bool = False,
         relu: bool = False, seq_t: int = 0, drop_seed: int = 0, drop_p: float = 0.0, drop_row0: int = 0,
         splits: int | None = None, a_hi: Sequence[torch.Tensor] | None = None, a_split: int = 0):
    """Batched C_i = alpha * op(A_i) op(B_i)^T (+bias) for up to 4 problems of one shape.
    With a_kouter and a_split > 0, A columns >= a_split are read from a_hi[i]."""
    nb = len(a)
    assert 1 <= nb <= 4 and len(b) == nb and len(c) == nb
    bt = GemmBatch()
    for i in range(nb):
        assert a[i].dtype == dtype and b[i].dtype == dtype, (a[i].dtype, b[i].dtype, dtype)
        assert c[i].dtype == out_dtype, (c[i].dtype, out_dtype)
        bt.a[i] = a[i].data_ptr()
        bt.b[i] = b[i].data_ptr()
        bt.c[i] = c[i].data_ptr()
        bt.bias[i] = bias[i].data_ptr() if bias is not None and bias[i] is not None else None
        bt.bshift[i] = bshift[i] if bshift is not None else 0
        if a_split:
            bt.a_hi[i] = a_hi[i].data_ptr()
    bt.a_split = a_split
    bt.drop_row0 = drop_row0 & 0xFFFFFFFF
    lib = _lib.load()
    if splits is None:
        splits = lib.tt_gemm_pick_splits(m, n, k, nb)
    ws = None
    if splits > 1 and not relu and drop_p == 0.0:
        ws = torch.empty(lib.tt_gemm_ws_size(m, n, nb, splits), dtype=torch.float32, device=c[0].device)
    else:
        splits = 1
    call("tt_gemm", dtype_code(dtype), dtype_code(out_dtype), int(a_kouter), int(b_kouter), m, n, k,
         ctypes.byref(bt), nb, lda, ldb, ldc, alpha, int(accumulate), int(relu), seq_t, drop_seed & 0xFFFFFFFF,
         drop_p, splits, ptr(ws), stream_ptr(c[0].device))


def embed_gather(table: torch.Tensor, ids: torch.Tensor, out: torch.Tensor):
    assert ids.dtype == torch.int32 and ids.is_contiguous()
    assert table.dim() == 2 and out.shape[-1] == table.shape[1] and out.dtype == table.dtype
    call("tt_embed_gather", dtype_code(table.dtype), table.data_ptr(), table.shape[0], table.shape[1],
         ids.data_ptr(), ids.numel(), out.data_ptr(), stream_ptr(out.device))


def pack_rows(src: torch.Tensor, out: torch.Tensor):
    assert src.dtype == torch.float32 and src.is_contiguous()
    e = src.shape[-1]
    n = src.numel() // e
    call("tt_pack_rows", dtype_code(out.dtype), src.data_ptr(), n, e, out.shape[-1], out.data_ptr(),
         stream_ptr(out.device))


def cast(x: torch.Tensor, out: torch.Tensor):
    assert x.dtype == torch.float32 and x.is_contiguous() and out.numel() == x.numel()
    call("tt_cast", dtype_code(out.dtype), x.data_ptr(), x.numel(), out.data_ptr(), stream_ptr(out.device))


def colsum(x: torch.Tensor, rows: int, cols: int, ld: int, out: torch.Tensor, accumulate: bool = False):
    assert x.dtype == torch.float32 and out.dtype == torch.float32
    call("tt_colsum", x.data_ptr(), rows, cols, ld, out.data_ptr(), int(accumulate), stream_ptr(out.device))


def total(x: torch.Tensor, scale: float, out: torch.Tensor):
    call("tt_sum", x.data_ptr(), x.numel(), scale, out.data_ptr(), stream_ptr(out.device))


def l2norm_fwd(x: torch.Tensor, eps: float, dt: torch.dtype, want_f32: bool = True):
    """Returns (y in dt, y32 fp32 or None, norm [rows])."""
    assert x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 2
    rows, cols = x.shape
    y = torch.empty(rows, cols, dtype=dt, device=x.device)
    y32 = y if dt == torch.float32 else (torch.empty_like(x) if want_f32 else None)
    norm = torch.empty(rows, dtype=torch.float32, device=x.device)
    call("tt_l2norm_fwd", dtype_code(dt), x.data_ptr(), rows, cols, eps, y.data_ptr(),
         None if y32 is y else ptr(y32), norm.data_ptr(), stream_ptr(x.device))
    return y, y32, norm


def l2norm_bwd(dy: torch.Tensor, y32: torch.Tensor, norm: torch.Tensor, eps: float, dx: torch.Tensor | None = None,
               accumulate: bool = False):
    assert dy.dtype == torch.float32 and dy.is_contiguous() and y32.dtype == torch.float32
    rows, cols = dy.shape
    if dx is None:
        dx = torch.empty_like(dy)
        accumulate = False
    call("tt_l2norm_bwd", dy.data_ptr(), y32.data_ptr(), norm.data_ptr(), rows, cols, eps, dx.data_ptr(),
         int(accumulate), stream_ptr(dy.device))
    return dx
