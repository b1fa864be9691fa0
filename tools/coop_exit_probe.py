"""Diagnostic for the exit-time SIGSEGV seen under rocprofv3 with the cooperative launch of
the column-split GRU forward (option gru_xc_coop = 1; DESIGN.md §12, verdict round 5 item 7).

Runs bench.py in this process after registering an atexit hook that copies /proc/self/maps
to OUT (Python's atexit hooks run before the C-level exit handlers and static destructors,
where the fault happens), so the faulting PC and the stack frames of the crash report can be
mapped to (library, offset) and symbolised offline with llvm-symbolizer against the same
ROCm image.

    rocprofv3 --kernel-trace --stats -d gpurun_out/X -- python tools/coop_exit_probe.py OUT bench-args...
"""
import atexit
import os
import runpy
import shutil
import sys

OUT = sys.argv[1]


def _dump():
    try:
        shutil.copyfile("/proc/self/maps", OUT)
        print(f"coop_exit_probe: maps -> {OUT}", file=sys.stderr, flush=True)
    except OSError as e:
        print(f"coop_exit_probe: {e}", file=sys.stderr, flush=True)


atexit.register(_dump)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
