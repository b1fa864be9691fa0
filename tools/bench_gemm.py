"""Micro-benchmark of tt_gemm on the step's GEMM shapes (HIP-event timed)."""
import argparse
import json
import sys

import torch

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from two_towers_amd import ops  # noqa: E402

SHAPES = {  # name: (m, n, k, a_kouter, b_kouter, nbatch, out_bf16)
    "input_proj_l1": (524288, 3072, 1024, 0, 0, 2, 1),
    "input_proj_l0": (524288, 3072, 320, 0, 0, 2, 1),  # Ep 320 since round 2 (304 before)
    "dgrad_l1": (524288, 1024, 3072, 0, 1, 1, 1),
    "wgrad_ih1": (1536, 1024, 524288, 1, 1, 4, 0),
    "wgrad_ih0": (1536, 320, 524288, 1, 1, 4, 0),  # N = Ep 320: two 256-column tiles, the second a quarter full
    "wgrad_hh": (1536, 512, 524288, 1, 1, 4, 0),
    "square8k": (8192, 8192, 8192, 0, 0, 1, 1),
    # diagnostics: the round-1 16-byte padding; the l1 FLOPs with a B small enough for L2
    "input_proj_l0_k304": (524288, 3072, 304, 0, 0, 2, 1),
    "proj_l1_n768": (2097152, 768, 1024, 0, 0, 2, 1),
    "sq_k1024": (16384, 16384, 1024, 0, 0, 1, 1),
    # configs[4] (H 1024, T 128, B 8192): input projection l1 and dX l1
    "c4_proj_l1": (1048576, 6144, 2048, 0, 0, 2, 1),
    "c4_dgrad_l1": (1048576, 2048, 6144, 0, 1, 1, 1),
}
# K sweep at the input-projection M/N (persistent kernel up to 24 K-tiles): separates the
# per-tile cost from the per-K-tile cost
for _k in (128, 192, 320, 512, 768, 1024, 1536):
    SHAPES[f"proj_k{_k}"] = (524288, 3072, _k, 0, 0, 2, 1)


NO_BIAS = False


def run(name, iters, lda_pad=0):
    m, n, k, ak, bk, nb, obf = SHAPES[name]
    dt = torch.bfloat16
    if lda_pad < 0 and not ak:  # every A row the same 16 KiB-or-less row (lda 0): A from L2
        A = [torch.randn(1, k, device="cuda").to(dt) for _ in range(nb)]
    elif lda_pad and not ak:  # A rows lda_pad elements apart (a strided view)
        A = [torch.randn(m, lda_pad, device="cuda").to(dt)[:, :k] for _ in range(nb)]
    else:
        A = [torch.randn((k, m) if ak else (m, k), device="cuda").to(dt) for _ in range(nb)]
    B = [torch.randn((k, n) if bk else (n, k), device="cuda").to(dt) for _ in range(nb)]
    odt = dt if obf else torch.float32
    C = [torch.empty(m, n, device="cuda", dtype=odt) for _ in range(nb)]
    bias = [torch.randn(n, device="cuda") for _ in range(nb)] if obf and not NO_BIAS else None
    f = lambda: ops.gemm(A, B, C, m=m, n=n, k=k, lda=m if ak else (0 if lda_pad < 0 else (lda_pad or k)), ldb=n if bk else k, ldc=n, a_kouter=bool(ak),
                         b_kouter=bool(bk), dtype=dt, out_dtype=odt, bias=bias)
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    tf = 2.0 * m * n * k * nb / (ms * 1e-3) / 1e12
    return {"shape": name, "ms": round(ms, 3), "tflops": round(tf, 1)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--regstage", default="", help="TT_GEMM_REGSTAGE value (9 = no epilogue, timing only)")
    ap.add_argument("--lda-pad", type=int, default=0, help="A row stride in elements (K-contig A); -1: lda 0, one row")
    ap.add_argument("--variants", default="", help="';'-separated option sets, each 'name=v,name=v' (tt_set_option); "
                                                   "'-' = defaults; rounds interleave the variants")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--no-bias", action="store_true", help="no bias epilogue (e.g. option gemm_il)")
    a = ap.parse_args()
    NO_BIAS = a.no_bias
    if a.regstage:
        os.environ["TT_GEMM_REGSTAGE"] = a.regstage
    if not a.variants:
        for nm in a.shapes.split(","):
            print(json.dumps(run(nm, a.iters, a.lda_pad)), flush=True)
    else:
        from two_towers_amd._lib import get_option, set_option
        sets = [v for v in a.variants.split(";") if v]
        names = sorted({kv.split("=")[0] for v in sets if v != "-" for kv in v.split(",")})
        dflt = {n: get_option(n) for n in names}
        for rnd in range(a.rounds):
            for v in sets:
                opts = dict(dflt)
                if v != "-":
                    opts.update({kv.split("=")[0]: int(kv.split("=")[1]) for kv in v.split(",")})
                for n, x in opts.items():
                    set_option(n, x)
                for nm in a.shapes.split(","):
                    r = run(nm, a.iters, a.lda_pad)
                    r.update(variant=v, round=rnd)
                    print(json.dumps(r), flush=True)
