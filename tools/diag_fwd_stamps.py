"""Per-phase breakdown of the persistent GRU forward (gru_fwd_seq) from s_memtime stamps
of wave 0 of every workgroup. Needs the diagnostic build (-DTT_DIAG, which exports
tt_diag_fwd_prof): TT_HIP_LIB=.../libtt_hip_diag.so python tools/diag_fwd_stamps.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from two_towers_amd import _lib  # noqa: E402
from two_towers_amd._lib import call, stream_ptr  # noqa: E402
import bench_gru  # noqa: E402  (tools/ on sys.path: same directory)

NAMES = ["kstep: W_hh issue + LDS frags + MFMA", "kstep: ring wait + W_hh LDS store", "kstep: barrier",
         "epi: gate staging + barrier", "epi: gate math + stores issued", "-", "-", "total"]


def main():
    B, T, H = 8192, 64, 512
    dev = torch.device("cuda")
    recs, keep = bench_gru.setup(B, T, H, dev)
    st = stream_ptr(dev)
    f = lambda: call("tt_gru_fwd", 1, recs, 4, B, T, H, 6 * H, 2 * H, 0.1, st)
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    f()
    e.record()
    torch.cuda.synchronize()
    lib = _lib.load()
    buf = np.zeros((2048, 8), dtype=np.uint64)
    lib.tt_diag_fwd_prof.restype = ctypes.c_int
    assert lib.tt_diag_fwd_prof(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    nwg = (B // 64) * 4
    p = buf[:nwg].astype(np.float64)
    tot = p[:, 7].mean()
    out = {"ms": round(s.elapsed_time(e), 3), "workgroups": nwg, "cycles_total_per_wg": round(tot)}
    for i, n in enumerate(NAMES):
        if n != "-" and i != 7:
            out[n] = round(float(p[:, i].mean() / tot), 3)
    out["unaccounted (h update, loop overhead)"] = round(1 - sum(float(p[:, i].mean()) for i in range(5)) / tot, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
