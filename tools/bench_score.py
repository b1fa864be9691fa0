"""Micro-benchmark of the score-matrix kernels at the bench shapes (HIP-event timed on
the launching stream): hard-negative mining (tt_hardneg_topk) and the fused InfoNCE
forward. Run under `rocprofv3 --kernel-trace --stats` for the per-kernel split."""
import argparse
import contextlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from two_towers_amd import _lib  # noqa: E402
from two_towers_amd._lib import call, dtype_code  # noqa: E402


def timed(f, iters):
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def hardneg(B, nd, h, k, dt, iters, flush_mb=0):
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(5)
    q = torch.nn.functional.normalize(torch.randn(B, h, device="cuda", generator=g), dim=1).to(dt)
    d = torch.nn.functional.normalize(torch.randn(nd, h, device="cuda", generator=g), dim=1).to(dt)
    idx = torch.empty(B, k, dtype=torch.int32, device="cuda")
    ws = torch.empty(lib.tt_hardneg_ws_size(dtype_code(dt), B, nd, h, k), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: call("tt_hardneg_topk", dtype_code(dt), q.data_ptr(), B, d.data_ptr(), nd, h, 0, k, idx.data_ptr(),
                     None, ws.data_ptr(), st)
    if flush_mb:  # a copy of flush_mb MiB before every call evicts the L2s and the MALL (the event time
        # then includes the copy: read the scan's own duration from a kernel trace)
        src = torch.empty(flush_mb << 20, dtype=torch.uint8, device="cuda")
        dst = torch.empty_like(src)
        f0 = f
        f = lambda: (dst.copy_(src), f0())
    ms = timed(f, iters)
    tf = 2.0 * B * nd * h / (ms * 1e-3) / 1e12
    return {"op": "hardneg_topk", "B": B, "nd": nd, "h": h, "k": k, "dtype": str(dt)[6:], "ms": round(ms, 4),
            "tflops": round(tf, 1), "mfma_frac": round(tf / 2500.0, 4)}


def infonce(B, nd, h, dt, iters):
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(6)
    q = torch.nn.functional.normalize(torch.randn(B, h, device="cuda", generator=g), dim=1).to(dt)
    d = torch.nn.functional.normalize(torch.randn(nd, h, device="cuda", generator=g), dim=1).to(dt)
    lse = torch.empty(B, device="cuda")
    rl = torch.empty(B, device="cuda")
    ws = torch.empty(max(lib.tt_infonce_fwd_ws_size(B, nd), 1), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: call("tt_infonce_fwd", dtype_code(dt), q.data_ptr(), B, d.data_ptr(), nd, h, 1.0 / 0.07, 0.0, 0,
                     lse.data_ptr(), rl.data_ptr(), ws.data_ptr(), st)
    ms = timed(f, iters)
    tf = 2.0 * B * nd * h / (ms * 1e-3) / 1e12
    f()
    dq = torch.empty(B, h, device="cuda")
    dd = torch.empty(nd, h, device="cuda")
    gs = torch.tensor([1.0 / B], device="cuda")
    for flash in (1, 0):  # fused (no dS) vs materialised dS
        with _lib.option("infonce_flash", flash):
            wsb = torch.empty(max(lib.tt_infonce_bwd_ws_size(dtype_code(dt), B, nd, h), 1), dtype=torch.uint8,
                              device="cuda")
            fb = lambda: call("tt_infonce_bwd", dtype_code(dt), q.data_ptr(), B, d.data_ptr(), nd, h, 1.0 / 0.07,
                              0.0, 0, lse.data_ptr(), gs.data_ptr(), dq.data_ptr(), dd.data_ptr(), wsb.data_ptr(), st)
            msb = timed(fb, iters)
        tfb = 6.0 * B * nd * h / (msb * 1e-3) / 1e12
        print(json.dumps({"op": "infonce_bwd", "flash": flash, "B": B, "nd": nd, "h": h, "dtype": str(dt)[6:],
                          "ms": round(msb, 4), "ws_bytes": wsb.numel(), "tflops": round(tfb, 1),
                          "mfma_frac": round(tfb / 2500.0, 4)}), flush=True)
        del wsb
    return {"op": "infonce_fwd", "B": B, "nd": nd, "h": h, "dtype": str(dt)[6:], "ms": round(ms, 4),
            "tflops": round(tf, 1), "mfma_frac": round(tf / 2500.0, 4)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ops", default="hardneg,infonce")
    ap.add_argument("--hn-shapes", default="8192x8192x256,8192x65536x256,8192x8192x512",
                    help="hard-negative shapes B x N x h")
    ap.add_argument("--flush-mb", type=int, default=0, help="copy this many MiB before every hard-negative call")
    ap.add_argument("--variants", default="", help='hard-negative option sets, e.g. "wide=hn_wide=1;map=hn_map=1"')
    a = ap.parse_args()
    bf = torch.bfloat16
    variants = [("default", {})]
    for v in filter(None, a.variants.split(";")):
        name, rest = v.split("=", 1)
        variants.append((name, {kv.split("=")[0]: int(kv.split("=")[1]) for kv in rest.split(",")}))
    if "hardneg" in a.ops:
        for shp in a.hn_shapes.split(","):
            B, nd, h = (int(x) for x in shp.split("x"))
            for name, opts in variants:
                with contextlib.ExitStack() as es:
                    for k, v in opts.items():
                        es.enter_context(_lib.option(k, v))
                    r = hardneg(B, nd, h, 5, bf, a.iters, a.flush_mb)
                r["variant"] = name
                print(json.dumps(r), flush=True)
    if "infonce" in a.ops:
        for B, nd, h in ((8192, 8192, 256), (8192, 65536, 256), (8192, 8192, 512)):
            print(json.dumps(infonce(B, nd, h, bf, a.iters)), flush=True)
