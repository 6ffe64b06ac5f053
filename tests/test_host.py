"""Host side, no GPU: the C ABI library's exports, the C++ driver's hashers,
generators and JSON output, and the phjoin CLI's argument handling."""
import ctypes
import json
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
PKG = os.path.join(ROOT, "partitionedhashjoin_amd")
LIB = os.path.join(PKG, "libphj_hip.so")
CLI = os.path.join(PKG, "phjoin")


def header_symbols():
    with open(os.path.join(ROOT, "include", "phj.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(phj_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build first: make / __graft_entry__.build()"
    lib = ctypes.CDLL(LIB)   # loads on a GPU-less host; no compute call is made
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    from partitionedhashjoin_amd import _capi
    assert sorted(_capi.EXPORTED) == syms
    assert lib.phj_abi_version() == _capi.ABI_VERSION == 2


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    import partitionedhashjoin_amd as phj
    with pytest.raises(phj.PhjError):
        phj.Context(0)


def test_struct_layouts():
    from partitionedhashjoin_amd import _capi
    assert ctypes.sizeof(_capi.Tuple) == 16
    assert ctypes.sizeof(_capi.JoinParams) == 32
    assert ctypes.sizeof(_capi.Partitioned) == 40


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("hc") / "host_check")
    srcs = [os.path.join(ROOT, "tests", "host", "host_check.cpp"),
            os.path.join(PKG, "host", "DataGenerator", "Generators.cpp"),
            os.path.join(PKG, "host", "Common", "Common.cpp")]
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-pthread", "-ffp-contract=off",
                           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "host"),
                           "-I" + os.path.join(PKG, "csrc"), "-o", exe] + srcs)
    return exe


def run(exe, *args):
    return subprocess.run([exe] + [str(a) for a in args], check=True, capture_output=True, text=True).stdout


def test_host_hashers_match_golden(host_check):
    for name in ("xxh3", "murmur3"):
        with open(os.path.join(GOLD, f"{name}.json")) as f:
            vecs = json.load(f)["vectors"]
        for v in vecs[::7]:
            h, hm = run(host_check, "hash", name, v["key"], v["seed"]).split()
            assert int(h) == v["hash"]
            assert int(hm) == v["hash"] % 1000


def test_host_generators_match_reference_outputs(host_check):
    with open(os.path.join(GOLD, "generators.json")) as f:
        gen = json.load(f)
    for g in gen["fill_zipf"]:
        n = g["batches"] * O.GEN_BATCH
        out = np.array(run(host_check, "zipf", g["alpha"], g["lo"], g["hi"], g["seed"], n).split(),
                       dtype=np.int64).reshape(-1, 2)
        assert out[:, 0].tolist() == g["ids"]
        assert out[:, 1].tolist() == g["payloads"]
    g = gen["fill_sequential"][0]
    out = np.array(run(host_check, "seq", g["start"], g["n"]).split(), dtype=np.int64).reshape(-1, 2)
    assert out[:8, 0].tolist() == g["ids_head"] and out[-8:, 0].tolist() == g["ids_tail"]
    # and the host generator equals the oracle's restatement on a ragged size
    n = 3 * O.GEN_BATCH + 17
    out = np.array(run(host_check, "zipf", 1.25, 1, 5000, 99, n).split(), dtype=np.int64).reshape(-1, 2)
    assert np.array_equal(out, O.fill_zipf(n, 1.25, 1, 5000, 99))


@pytest.mark.parametrize("fixture,args", [
    ("partitions_256_s1.05.txt", ("ms", "RadixParitioning", 256, 10000000, 200000000, 1.05,
                                  729_000_000, 29_000_000, 456_000_000)),
    ("partitions_1_s1.05.txt", ("ms", "NoPartitioning", "-", 10000000, 200000000, 1.05,
                                0, 308_000_000, 1112_000_000)),
    ("partitions_1_s1.25.txt", ("ms", "NoPartitioning", "-", 10000000, 200000000, 1.25,
                                0, 310_000_000, 691_000_000)),
])
def test_json_output_is_byte_compatible_with_reference_results(host_check, fixture, args):
    # the reference's own published result files (results/*/partitions_*.txt)
    with open(os.path.join(GOLD, "reference_results", fixture)) as f:
        expect = f.read()
    assert run(host_check, "json", *args) == expect


def test_json_units(host_check):
    out = json.loads(run(host_check, "json", "us", "NoPartitioning", "-", 1, 2, 1.05, 0, 1500, 2_500_000))
    assert out["results"] == {"partition": "0", "build": "1", "probe": "2500"}
    assert out["parameters"]["Skew"] == "1.050000"


def cli(*args):
    return subprocess.run([CLI] + list(args), capture_output=True, text=True, cwd="/tmp")


def test_cli_help():
    r = cli("--help")
    assert r.returncode == 0 and "--join" in r.stdout and "--partitions" in r.stdout


@pytest.mark.parametrize("args,msg", [
    ((), "--join' is required"),
    (("--join", "hash"), "Unrecognized join algorithm type"),
    (("--join", "no-partitioning", "-p", "64"), "number of partitions can be specified only for RadixParitioning"),
    (("--join", "radix-partitioning", "-u", "hours"), "Unrecognized time unit"),
    (("--join", "radix-partitioning", "--format", "xml"), "Unrecognized results format"),
    (("--join", "radix-partitioning", "-o", "socket"), "Unrecognized output type"),
    (("--join", "radix-partitioning", "--primary", "ten"), "is invalid"),
    (("--join", "radix-partitioning", "--bogus", "1"), "unrecognised option"),
    (("--join", "radix-partitioning", "--radix-bits", "12"), "1..11 bits"),
])
def test_cli_validation(args, msg):
    # parse errors print the message and the help, then exit(1) (src/main.cpp:201-205)
    r = cli(*args)
    assert r.returncode == 1
    assert msg in r.stdout


def test_cli_without_gpu_exits_1(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    r = subprocess.run([CLI, "--join", "radix-partitioning", "--primary", "1000", "--secondary", "10000",
                        "-f", str(tmp_path / "out.txt")], capture_output=True, text=True)
    assert r.returncode == 1
    assert "No usable HIP device" in r.stderr


def test_join_path_declines_lds_join_above_the_pool_bound():
    """the LDS join needs the probe side's keys-only chunked
    pass 1, whose chunk pools address slots with 32 bits. Above that bound
    (about 1.07e9 probe rows with the pipelined pass's reservations) the join
    must take the code tables (the stable pass 1 and k_probe_ht), not fail.
    Host-only (phj_join_path: the decision phj_join makes, no device)."""
    import partitionedhashjoin_amd as phj
    c2 = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3)
    nR = 10_000_000
    assert phj.join_path(c2, nR, 200_000_000) == phj.PATH_LDS_JOIN
    assert phj.join_path(c2, nR, 0) == phj.PATH_LDS_JOIN
    # the largest probe side the LDS join takes, found by bisection, then the
    # rows just above it: every size up to the per-device limit has a path
    lo, hi = 200_000_000, (1 << 32) - 2 * 4096 - 1
    assert phj.join_path(c2, nR, hi) == phj.PATH_CODE_TABLES
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if phj.join_path(c2, nR, mid) == phj.PATH_LDS_JOIN:
            lo = mid
        else:
            hi = mid
    assert 0.5e9 < lo < 2.2e9
    assert phj.join_path(c2, nR, lo + 1) == phj.PATH_CODE_TABLES
    # the reference's own -p plans, stable layouts and NoPartitioning
    assert phj.join_path(phj.radix_params(num_partitions=1024, hash=phj.HASH_XXH3), nR, 200_000_000) == phj.PATH_LDS_JOIN
    assert phj.join_path(phj.radix_params((8, 8), stable=True), nR, 1000) != phj.PATH_LDS_JOIN
    assert phj.join_path(phj.nopart_params(), nR, 200_000_000) == phj.PATH_NO_PARTITIONING
