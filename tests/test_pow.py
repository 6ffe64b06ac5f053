"""The device Zipf generator's pow (csrc/phj_pow.h) against this host's glibc
pow, compiled for the host: the FMA restatement must agree bit for bit on the
generator's own calls (Zipf.cpp:29-50 at several skews and cardinalities) and
on random finite arguments. Also: the committed table header is exactly what
scripts/gen_pow_tables.py reads from libm."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "partitionedhashjoin_amd", "csrc")


def test_pow_restatement_matches_host_glibc(tmp_path):
    exe = tmp_path / "pow_check"
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-ffp-contract=off", f"-I{CSRC}", "-o", str(exe),
                           os.path.join(ROOT, "tests", "host", "pow_check.cpp")])
    out = subprocess.run([str(exe), "3000000"], capture_output=True, text=True, check=True).stdout
    res = {line.split()[0]: (int(line.split()[1]), int(line.split()[2])) for line in out.splitlines()}
    bad, total = res["fma"]
    assert total > 10_000_000
    assert bad == 0, out


@pytest.mark.skipif(not os.path.exists("/lib/x86_64-linux-gnu/libm.so.6"), reason="no glibc libm")
def test_pow_tables_are_libm_tables(tmp_path):
    out = tmp_path / "t.h"
    subprocess.check_call(["python3", os.path.join(ROOT, "scripts", "gen_pow_tables.py"), str(out)])
    with open(os.path.join(CSRC, "phj_pow_tables.h")) as f:
        assert f.read() == out.read_text()
