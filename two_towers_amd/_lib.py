"""ctypes binding of libtt_hip.so (the C ABI declared in include/tt_hip.h).

This module is the only place that touches the shared library. There is no CPU
fallback: if the library is missing or no ROCm GPU is visible, every op raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from ctypes import POINTER, c_float, c_int, c_long, c_uint32, c_void_p

import torch  # must be imported first so libtt_hip.so binds torch's HIP runtime

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TT_HIP_LIB", os.path.join(_HERE, "lib", "libtt_hip.so"))

DT_F32 = 0
DT_BF16 = 1
TT_EINVAL = 1000


class TTError(RuntimeError):
    pass


class GruTimeoutError(TTError):
    """A column-split GRU forward launch gave up waiting for one of its member workgroups
    (tt_gru_fwd's status word): that launch's outputs are invalid."""


class GemmBatch(ctypes.Structure):
    _fields_ = [
        ("a", c_void_p * 4),
        ("b", c_void_p * 4),
        ("c", c_void_p * 4),
        ("bias", c_void_p * 4),
        ("bshift", c_int * 4),
        ("a_hi", c_void_p * 4),
        ("a_split", c_int),
        ("drop_row0", c_uint32),
    ]


class PackJob(ctypes.Structure):  # include/tt_hip.h tt_pack_job
    _fields_ = [
        ("src", c_void_p),
        ("src2", c_void_p),
        ("dst", c_void_p),
        ("rows", c_int),
        ("cols", c_int),
        ("dcols", c_int),
        ("lds", c_long),
        ("ldd", c_long),
        ("dst_bf16", c_int),
    ]


class GruFwdRec(ctypes.Structure):
    _fields_ = [
        ("g", c_void_p), ("whh", c_void_p), ("bhn", c_void_p), ("y", c_void_p), ("x1", c_void_p),
        ("save", c_void_p), ("hstate", c_void_p), ("dir", c_int), ("drop_seed", c_uint32),
        ("drop_col0", c_int), ("drop_row0", c_uint32),
    ]


class GruBwdRec(ctypes.Structure):
    _fields_ = [
        ("save", c_void_p), ("y", c_void_p), ("dy", c_void_p), ("dfinal", c_void_p), ("whh", c_void_p),
        ("dgx", c_void_p), ("dgh", c_void_p), ("dhstate", c_void_p), ("dbias_part", c_void_p),
        ("dir", c_int),
    ]


class HeadFwdIO(ctypes.Structure):
    _fields_ = [
        ("w1", c_void_p), ("b1", c_void_p), ("ln_g", c_void_p), ("ln_b", c_void_p), ("w2", c_void_p),
        ("b2", c_void_p), ("x", c_void_p), ("p1", c_void_p), ("mean", c_void_p), ("rstd", c_void_p),
        ("u", c_void_p), ("out", c_void_p),
    ]


class HeadBwdIO(ctypes.Structure):
    _fields_ = [
        ("w1", c_void_p), ("ln_g", c_void_p), ("ln_b", c_void_p), ("w2", c_void_p), ("x", c_void_p),
        ("p1", c_void_p), ("mean", c_void_p), ("rstd", c_void_p), ("u", c_void_p), ("dout", c_void_p),
        ("dx", c_void_p), ("dw1", c_void_p), ("db1", c_void_p), ("dg", c_void_p), ("dbeta", c_void_p),
        ("dw2", c_void_p), ("db2", c_void_p), ("ws", c_void_p),
    ]


class Head1FwdIO(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("w1", c_void_p), ("b1", c_void_p), ("ln_g", c_void_p), ("ln_b", c_void_p),
        ("p1", c_void_p), ("mean", c_void_p), ("rstd", c_void_p), ("out", c_void_p),
    ]


class Head1BwdIO(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("w1", c_void_p), ("ln_g", c_void_p), ("ln_b", c_void_p), ("p1", c_void_p),
        ("mean", c_void_p), ("rstd", c_void_p), ("dout", c_void_p), ("dx", c_void_p), ("dw1", c_void_p),
        ("db1", c_void_p), ("dg", c_void_p), ("dbeta", c_void_p), ("ws", c_void_p),
    ]


# name -> (restype, argtypes). Kept in the order of include/tt_hip.h.
_SIGS = {
    "tt_version": (ctypes.c_char_p, []),
    "tt_last_error": (ctypes.c_char_p, []),
    "tt_set_option": (c_int, [ctypes.c_char_p, c_int]),
    "tt_get_option": (c_int, [ctypes.c_char_p, POINTER(c_int)]),
    "tt_embed_gather": (c_int, [c_int, c_void_p, c_long, c_int, c_void_p, c_long, c_void_p, c_void_p]),
    "tt_pack_rows": (c_int, [c_int, c_void_p, c_long, c_int, c_int, c_void_p, c_void_p]),
    "tt_pack_multi": (c_int, [c_void_p, c_int, c_void_p]),
    "tt_cast": (c_int, [c_int, c_void_p, c_long, c_void_p, c_void_p]),
    "tt_colsum": (c_int, [c_void_p, c_long, c_int, c_long, c_void_p, c_int, c_void_p]),
    "tt_gemm": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, POINTER(GemmBatch), c_int, c_long,
                        c_long, c_long, c_float, c_int, c_int, c_int, c_uint32, c_float, c_int, c_void_p,
                        c_void_p]),
    "tt_gemm_ws_size": (c_long, [c_int, c_int, c_int, c_int]),
    "tt_gemm_pick_splits": (c_int, [c_int, c_int, c_int, c_int]),
    "tt_gru_fwd": (c_int, [c_int, POINTER(GruFwdRec), c_int, c_int, c_int, c_int, c_long, c_long, c_float,
                           c_void_p, c_long, c_void_p]),
    "tt_gru_bwd": (c_int, [c_int, POINTER(GruBwdRec), c_int, c_int, c_int, c_int, c_long, c_long, c_long,
                           c_void_p]),
    "tt_gru_bias_rows": (c_int, [c_int]),
    "tt_gru_bwd_launches": (c_int, [c_int, c_int, c_int]),
    "tt_gru_bwd_carry_on_chip": (c_int, [c_int, c_int, c_int]),
    "tt_gru_fwd_launches": (c_int, [c_int, c_int, c_int]),
    "tt_gru_fwd_ws_size": (c_long, [c_int, c_int, c_int, c_int, c_int, c_long, c_long]),
    "tt_gru_fwd_launches_for": (c_int, [c_int, c_int, c_int, c_int, c_int, c_long, c_long]),
    "tt_proj_head_fwd": (c_int, [c_int, POINTER(HeadFwdIO), c_int, c_int, c_int, c_float, c_void_p]),
    "tt_proj_head_bwd": (c_int, [c_int, POINTER(HeadBwdIO), c_int, c_int, c_int, c_float, c_void_p]),
    "tt_proj_head_bwd_ws_size": (c_long, [c_int, c_int, c_int]),
    "tt_proj_head1_fwd": (c_int, [c_int, POINTER(Head1FwdIO), c_long, c_int, c_float, c_float, c_uint32,
                                  c_void_p]),
    "tt_proj_head1_bwd": (c_int, [c_int, POINTER(Head1BwdIO), c_long, c_int, c_float, c_uint32, c_void_p]),
    "tt_proj_head1_bwd_ws_size": (c_long, [c_int, c_long, c_int]),
    "tt_l2norm_fwd": (c_int, [c_int, c_void_p, c_long, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "tt_l2norm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_long, c_int, c_float, c_void_p, c_int, c_void_p]),
    "tt_infonce_fwd": (c_int, [c_int, c_void_p, c_long, c_void_p, c_long, c_int, c_float, c_float, c_long,
                               c_void_p, c_void_p, c_void_p, c_void_p]),
    "tt_infonce_fwd_ws_size": (c_long, [c_long, c_long]),
    "tt_infonce_bwd": (c_int, [c_int, c_void_p, c_long, c_void_p, c_long, c_int, c_float, c_float, c_long,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "tt_infonce_bwd_ws_size": (c_long, [c_int, c_long, c_long, c_int]),
    "tt_hardneg_topk": (c_int, [c_int, c_void_p, c_long, c_void_p, c_long, c_int, c_long, c_int, c_void_p,
                                c_void_p, c_void_p, c_void_p]),
    "tt_hardneg_ws_size": (c_long, [c_int, c_long, c_long, c_int, c_int]),
    "tt_search_topk": (c_int, [c_int, c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_void_p, c_void_p,
                               c_void_p, c_void_p]),
    "tt_search_ws_size": (c_long, [c_int, c_long, c_long, c_int, c_int]),
    "tt_margin_fwd": (c_int, [c_void_p, c_long, c_void_p, c_long, c_int, c_long, c_void_p, c_int, c_float,
                              c_void_p, c_void_p]),
    "tt_margin_bwd": (c_int, [c_void_p, c_long, c_void_p, c_long, c_int, c_long, c_void_p, c_int, c_float,
                              c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "tt_margin_bwd_ws_size": (c_long, [c_long, c_long, c_int, c_int]),
    "tt_sum": (c_int, [c_void_p, c_long, c_float, c_void_p, c_void_p]),
    "tt_adam_multi": (c_int, [POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p),
                              POINTER(c_long), c_int, c_float, c_float, c_float, c_float, c_float, c_int,
                              c_void_p, c_void_p]),
}

EXPORTED = tuple(_SIGS)

_lib = None
_load_error: str | None = None


def load():
    """Load libtt_hip.so once; raise TTError (never fall back) if it cannot be loaded."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise TTError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"two_towers_amd: native library not found at {LIB_PATH}; "
                       "build it with `python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        raise TTError(_load_error)
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = _lib.tt_last_error().decode(errors="replace") if _lib is not None else ""
        raise TTError(f"{what or 'tt_hip'} failed (rc={rc}): {msg}")


def call(name: str, *args):
    lib = load()
    check(getattr(lib, name)(*args), name)


def get_option(name: str) -> int:
    v = c_int(0)
    call("tt_get_option", name.encode(), ctypes.byref(v))
    return v.value


def set_option(name: str, value: int) -> int:
    """Select a kernel variant (tt_set_option); returns the previous value."""
    old = get_option(name)
    call("tt_set_option", name.encode(), int(value))
    return old


@contextlib.contextmanager
def option(name: str, value: int):
    """with option("gru_step", 1): ...  -- a variant for the duration of the block."""
    torch.cuda.synchronize()
    old = set_option(name, value)
    try:
        yield
    finally:
        torch.cuda.synchronize()
        set_option(name, old)


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(*tensors: torch.Tensor):
    """The product path runs only on a ROCm GPU through libtt_hip.so."""
    load()
    for t in tensors:
        if t is not None and t.device.type != "cuda":
            raise TTError(
                "two_towers_amd runs only on an AMD GPU (HIP, gfx950); got a tensor on "
                f"'{t.device}'. There is deliberately no CPU fallback: move the model and "
                "inputs to the GPU (`.to('cuda')`).")


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return DT_F32
    if dt == torch.bfloat16:
        return DT_BF16
    raise TTError(f"unsupported compute dtype {dt}; use torch.float32 or torch.bfloat16")
