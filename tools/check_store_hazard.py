#!/usr/bin/env python3
"""Scan gfx950 device code for the wide-buffer-store data hazard that corrupted the
persistent GRU forward's saved gh_n in round 2 ("root cause").

A `buffer_store_dwordx3/x4` reads its data VGPRs after issue; a VALU instruction that
overwrites one of them within the next two wait states can replace part of the stored
data (the lanes whose data is read last). LLVM inserts the wait states for this hazard
only when the store's soffset is NOT a register (GCNHazardRecognizer::createsVALUHazard
exempts MUBUF stores with an SGPR soffset), so a store with an SGPR soffset followed at
once by a write of its data registers is emitted unprotected. That is exactly the
sequence found in gru_fwd_seq<1,0>:

    buffer_store_dwordx4 v[0:3], v158, s[40:43], s61 offen   ; gh_n, soffset = 6H bytes
    v_mov_b32_e32 v0, v22                                     ; fp32 y overwrites the data

This tool lists every wide buffer store with a register soffset (which the product code
must not contain any more: tt_common.h folds every store offset into voffset) and, among
them, every one whose data registers are rewritten within `--window` instructions.

Usage: python tools/check_store_hazard.py [two_towers_amd/lib/libtt_hip.so | file.s ...]
Exit status 1 if any wide store uses a register soffset.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
STORE = re.compile(r"^\s*(buffer_store_dwordx[34]|buffer_store_format_xyzw?|tbuffer_store_format_xyzw?)\s+(.*)$")
VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def vrange(op):
    m = VREG.match(op.strip())
    if not m:
        return None
    if m.group(1) is not None:
        n = int(m.group(1))
        return (n, n)
    return (int(m.group(2)), int(m.group(3)))


def disassemble(path):
    """Device disassembly text of a .so / code object, or the file itself if it is .s."""
    if path.endswith(".s"):
        return open(path).read()
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, os.path.basename(path))
        os.symlink(os.path.abspath(path), src)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", src], cwd=td, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        out = []
        for f in sorted(os.listdir(td)):
            if "amdgcn" in f:
                r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", os.path.join(td, f)],
                                   check=True, capture_output=True, text=True)
                out.append(r.stdout)
        if not out:  # a plain code object
            r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", path],
                               check=True, capture_output=True, text=True)
            out.append(r.stdout)
        return "\n".join(out)


def scan(text, window=2):
    func = "?"
    lines = text.splitlines()
    insts = []  # (func, text)
    for ln in lines:
        m = re.match(r"^([0-9a-f]+ )?<?([_A-Za-z][\w.$]*)>?:\s*(;.*)?$", ln.strip())
        if m and not ln.startswith("\t") and not ln.startswith(" "):
            func = m.group(2)
            continue
        s = ln.split("//")[0].split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        insts.append((func, s))
    reg_soff, hazards = [], []
    for i, (fn, s) in enumerate(insts):
        m = STORE.match(s)
        if not m:
            continue
        ops = [o.strip() for o in m.group(2).split(",")]
        # buffer_store_dwordx4 vdata, vaddr|off, s[rsrc], soffset [offen|idxen] [offset:N] ...
        if len(ops) < 4:
            continue
        soff = ops[3].split()[0]
        if not re.match(r"^(s\d+|s\[\d+:\d+\]|m0|vcc_lo|vcc_hi|ttmp\d+)$", soff):
            continue
        data = vrange(ops[0])
        reg_soff.append((fn, s))
        if data is None:
            continue
        waits = 0
        for fn2, s2 in insts[i + 1:i + 1 + 8]:
            if waits >= window:
                break
            mn = re.match(r"^s_nop\s+(\d+)", s2)
            if mn:
                waits += int(mn.group(1)) + 1
                continue
            if s2.startswith("v_"):
                dst = vrange(s2.split(None, 1)[1].split(",")[0]) if " " in s2 else None
                if dst and not (dst[1] < data[0] or dst[0] > data[1]):
                    hazards.append((fn, s, s2, waits))
                    break
            waits += 1
    return reg_soff, hazards


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="*", default=["two_towers_amd/lib/libtt_hip.so"])
    ap.add_argument("--window", type=int, default=2, help="wait states the hazard needs (gfx940+: 2)")
    args = ap.parse_args()
    bad = 0
    for p in args.paths:
        reg_soff, hazards = scan(disassemble(p), args.window)
        print(f"{p}: {len(reg_soff)} wide buffer stores with a register soffset, "
              f"{len(hazards)} with their data rewritten within {args.window} wait states")
        for fn, s, s2, w in hazards:
            print(f"  HAZARD in {fn}:\n    {s}\n    {s2}   (after {w} wait states)")
        funcs = sorted({fn for fn, _ in reg_soff})
        for fn in funcs:
            print(f"  register soffset in {fn}")
        bad += len(reg_soff)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
