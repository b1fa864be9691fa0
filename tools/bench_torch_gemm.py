"""torch.matmul (hipBLASLt) on the step's GEMM shapes, for a library reference point."""
import json

import torch

SHAPES = {  # name: (m, n, k, a_kouter, b_kouter, nbatch)
    "input_proj_l1": (524288, 3072, 1024, 0, 0, 2),
    "input_proj_l0": (524288, 3072, 320, 0, 0, 2),
    "dgrad_l1": (524288, 1024, 3072, 0, 1, 1),
    "wgrad_ih1": (1536, 1024, 524288, 1, 1, 4),
    "wgrad_hh": (1536, 512, 524288, 1, 1, 4),
    "square8k": (8192, 8192, 8192, 0, 0, 1),
}
for name, (m, n, k, ak, bk, nb) in SHAPES.items():
    dt = torch.bfloat16
    A = torch.randn((k, m) if ak else (m, k), device="cuda").to(dt)
    B = torch.randn((k, n) if bk else (n, k), device="cuda").to(dt)
    a = A.t() if ak else A
    b = B if bk else B.t()
    odt = torch.float32 if ak else dt
    f = lambda: torch.mm(a, b, out_dtype=odt) if odt != dt else torch.mm(a, b)
    try:
        f()
    except Exception:
        odt = dt
        f = lambda: torch.mm(a, b)
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 5
    s.record()
    for _ in range(it):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / it
    print(json.dumps({"shape": name, "ms_x1": round(ms, 3), "ms_batch": round(ms * nb, 3),
                      "tflops": round(2.0 * m * n * k / (ms * 1e-3) / 1e12, 1), "out": str(odt)}), flush=True)
