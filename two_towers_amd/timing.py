"""Optional live kernel timing with HIP events (used by bench.py).

Events are recorded on torch's current stream, which is the stream every libtt_hip
launch is issued on (the ops pass torch.cuda.current_stream()). A region records its
launch count and algorithmic work (FLOPs or bytes) so rooflines can be computed
from measured device time.
"""
from __future__ import annotations

from collections import defaultdict
from contextlib import contextmanager

import torch

enabled = False
_records = defaultdict(list)
_kernels = defaultdict(list)  # region -> kernel names it launched, in first-seen order


def reset():
    _records.clear()
    _kernels.clear()


@contextmanager
def region(name: str, launches: int, work: float, nbytes: float = 0.0, kernel: str | None = None):
    """work = algorithmic FLOPs (or bytes for pure data movement), nbytes =
    algorithmic HBM bytes of the region (inputs read once + outputs written once),
    kernel = the name of the kernel the region launches (as rocprofv3 prints it); a region
    entered with different kernels (the two GRU layers' instances) keeps every name."""
    if not enabled:
        yield
        return
    if kernel and kernel not in _kernels[name]:
        _kernels[name].append(kernel)
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    yield
    e.record()
    _records[name].append((s, e, launches, work, nbytes))


def summary():
    """name -> dict(ms_total, launches, work, ms_per_launch, work_per_launch). Synchronises."""
    torch.cuda.synchronize()
    out = {}
    for name, recs in _records.items():
        ms = sum(r[0].elapsed_time(r[1]) for r in recs)
        n = sum(r[2] for r in recs)
        w = sum(r[3] for r in recs)
        b = sum(r[4] for r in recs)
        out[name] = dict(ms_total=ms, launches=n, work=w, bytes=b, ms_per_launch=ms / max(n, 1),
                         work_per_launch=w / max(n, 1), bytes_per_launch=b / max(n, 1), calls=len(recs),
                         kernel=" | ".join(_kernels.get(name) or [name]), kernels=list(_kernels.get(name) or []))
    return out
