"""The inline-assembly loads of the hot kernels (the LDS join's codes) are
waited for by their own s_waitcnt: the compiled
device code must never touch a destination register before that wait
(scripts/check_asm_waits.py compiles the library to gfx950 assembly and scans
every such kernel). CPU only: hipcc cross-compiles."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="hipcc not available")
def test_no_register_touched_before_its_asm_wait():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_asm_waits.py")],
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    lines = p.stdout.splitlines()
    checked = [l for l in lines if "asm loads" in l]
    # the LDS join, tile and segment modes (S's pass 1 keeps the compiler's
    # waits: its inline-assembly form measured slower end to end)
    assert sum("k_cluster_probe" in l for l in checked) >= 2, p.stdout
