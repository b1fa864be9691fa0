"""Per-phase breakdown of the column-split GRU forward (gru_fwd_xc) from s_memtime stamps of
wave 0 of every workgroup, with the diagnostic switches of the -DTT_DIAG build (TT_GRU_DBG:
1 no group wait, 2 no Y / S / X1 stores, 4 no drain before the arrival count; the results
of 1 and 4 are wrong, for timing only).
TT_HIP_LIB=two_towers_amd/lib/libtt_hip_diag.so python tools/diag_xc.py [dbg ...]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from two_towers_amd import _lib  # noqa: E402
from two_towers_amd._lib import call, set_option, stream_ptr  # noqa: E402
import bench_gru  # noqa: E402

NAMES = ["wait + barrier", "prologue (h chunks 0-1, MFMA 0)", "chunk: MFMA + gates + restage issue",
         "chunk: barriers + staging", "drain + publish", "-", "-", "total"]


BWD_NAMES = ["wait + barrier", "prologue (chunks 0-1, MFMA 0)", "chunk: MFMA + gates + restage issue",
             "chunk: barriers + staging + partial sums", "drain + publish", "-", "-", "total"]


def main():
    B, T, H = 8192, 64, 512
    dev = torch.device("cuda")
    recs, keep = bench_gru.setup(B, T, H, dev)
    st = stream_ptr(dev)
    args = sys.argv[1:]
    bwd = bool(args) and args[0] == "bwd"
    if bwd:
        args = args[1:]
        call("tt_gru_fwd", 1, recs, 4, B, T, H, 6 * H, 2 * H, 0.1, st)
        brecs, bkeep = bench_gru.setup_bwd(B, T, H, keep, dev)
        set_option("gru_bwd_xc", 2)
        global NAMES
        NAMES = BWD_NAMES
    set_option("gru_fwd_xc", 2)
    lib = _lib.load()
    lib.tt_diag_fwd_prof.restype = ctypes.c_int
    for dbg in (args or ["0"]):
        os.environ["TT_GRU_DBG"] = dbg
        if bwd:
            f = lambda: call("tt_gru_bwd", 1, brecs, 4, B, T, H, 2 * H, 8 * H, 2 * H, st)
        else:
            f = lambda: call("tt_gru_fwd", 1, recs, 4, B, T, H, 6 * H, 2 * H, 0.1, st)
        f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        f()
        e.record()
        torch.cuda.synchronize()
        buf = np.zeros((2048, 8), dtype=np.uint64)
        assert lib.tt_diag_fwd_prof(buf.ctypes.data_as(ctypes.c_void_p)) == 0
        p = buf[:256].astype(np.float64)
        tot = p[:, 7].mean()
        out = {"dbg": dbg, "ms": round(s.elapsed_time(e), 3), "cycles_total_per_wg": round(tot)}
        for i, n in enumerate(NAMES):
            if n != "-" and i != 7:
                out[n] = round(float(p[:, i].mean() / tot), 3)
        print(json.dumps(out), flush=True)
        flag = ctypes.c_int(0)
        call("tt_gru_fwd_xc_status", ctypes.byref(flag))


if __name__ == "__main__":
    main()
