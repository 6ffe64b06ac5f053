#!/usr/bin/env python3
"""Static check of the kernels that issue loads by inline assembly with their
own s_waitcnt (k_cluster_probe's codes: csrc/phj_cluster.h ASMW).

The compiler does not know those loads are in flight: if it copied or read a
destination register between the load and the wait that covers it, the copy
would be taken before the data landed. This compiles the library's device code
to assembly (hipcc -S, gfx950) and, for every inline-assembly load, scans the
instructions after it up to the next inline-assembly s_waitcnt: none may touch
the load's destination registers (the scan follows program order; an
assembly s_waitcnt vmcnt(k) ends it once k vector-memory operations were
issued after the load). Prints one line per kernel; exit 1 on a hit.

  python scripts/check_asm_waits.py [--asm FILE.s]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "partitionedhashjoin_amd", "csrc", "phj_capi.hip")
LOAD = re.compile(r"(global_load_dwordx[24]|global_atomic_add)\s+(v\[?\d+(?::\d+)?\]?)")
REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")


def device_asm(out):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result", "-S",
                    "--offload-device-only", SRC, "-o", out], check=True, capture_output=True)


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    return set(range(int(m.group(1)), int(m.group(2)) + 1)) if m else {int(tok[1:])}


def kernels(lines):
    """(name, [lines]) of every function body."""
    name, body = None, []
    for l in lines:
        m = re.match(r"^([_A-Za-z0-9]+):\s*(;.*)?$", l)
        if m and not l.startswith(".") and m.group(1).startswith("_Z"):
            if name:
                yield name, body
            name, body = m.group(1), []
        elif name:
            body.append(l)
            if "s_endpgm" in l:
                yield name, body
                name, body = None, []


def check(body):
    """(asm loads, hits): hits = instructions touching an in-flight asm load's registers."""
    loads, inasm = [], False
    for i, l in enumerate(body):
        if "ASMSTART" in l:
            inasm = True
        elif "ASMEND" in l:
            inasm = False
        elif inasm:
            m = LOAD.search(l)
            if m:
                loads.append((i, m.group(2)))
    hits = []
    for li, tok in loads:
        R, inasm, after = regs(tok), False, 0
        for l in body[li + 1:]:
            if "ASMSTART" in l:
                inasm = True
                continue
            if "ASMEND" in l:
                inasm = False
                continue
            s = l.strip()
            if re.match(r"(global|buffer)_", s):
                after += 1   # vector-memory operations issued after the load (program order)
            w = re.search(r"s_waitcnt vmcnt\((\d+)\)", s)
            # an assembly wait for vmcnt(k) covers the load only when k operations
            # were issued after it on the way (else, e.g. a later tile's wait in
            # the unrolled loop, the scan goes on)
            if inasm and w and after >= int(w.group(1)):
                break
            if inasm or not s or s.startswith(";") or s.startswith("."):
                continue
            ops = s.split(None, 1)
            if len(ops) < 2:
                continue
            for m in REG.finditer(ops[1]):
                rr = set(range(int(m.group(1)), int(m.group(2)) + 1)) if m.group(1) else {int(m.group(3))}
                if rr & R:
                    hits.append((tok, s))
                    break
    return len(loads), hits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", help="an existing device assembly file (default: compile the library's)")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        path = a.asm or os.path.join(d, "dev.s")
        if not a.asm:
            device_asm(path)
        lines = open(path).read().split("\n")
    bad = checked = 0
    for name, body in kernels(lines):
        n, hits = check(body)
        if n == 0:
            continue
        checked += 1
        print(f"{name[:90]}: {n} asm loads, {len(hits)} touched before their wait")
        for tok, s in hits[:5]:
            print(f"    {tok}: {s}")
        bad += len(hits)
    print(f"kernels checked: {checked}, touches: {bad}")
    return 1 if bad or checked == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
