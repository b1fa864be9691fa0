"""Library GEMM rates (torch.matmul -> hipBLASLt on ROCm) on the step's GEMM shapes, beside
tools/bench_gemm.py's numbers for tt_gemm. Measurement only: nothing in the product path
calls it. Shapes as tools/bench_gemm.py (m, n, k, a_kouter, b_kouter, nbatch)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import SHAPES  # noqa: E402

NAMES = sys.argv[1].split(",") if len(sys.argv) > 1 else ["wgrad_ih1", "wgrad_hh", "dgrad_l1", "input_proj_l1",
                                                          "input_proj_l0", "square8k"]
for name in NAMES:
    m, n, k, ak, bk, nb, obf = SHAPES[name]
    dt = torch.bfloat16
    A = [torch.randn((k, m) if ak else (m, k), device="cuda").to(dt) for _ in range(nb)]
    B = [torch.randn((k, n) if bk else (n, k), device="cuda").to(dt) for _ in range(nb)]
    C = [torch.empty(m, n, device="cuda", dtype=dt) for _ in range(nb)]
    a_ = [x.t() if ak else x for x in A]
    b_ = [x if bk else x.t() for x in B]

    def f():
        for i in range(nb):
            torch.matmul(a_[i], b_[i], out=C[i])
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 5
    print(json.dumps({"shape": name, "lib": "torch.matmul", "ms": round(ms, 3),
                      "tflops": round(2.0 * m * n * k * nb / (ms * 1e-3) / 1e12, 1)}), flush=True)
