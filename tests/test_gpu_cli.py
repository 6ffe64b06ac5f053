"""The phjoin CLI end to end on the GPU: reference flags in, reference JSON
out, matched count equal to the oracle's on the same (seeded) relations."""
import json
import os
import subprocess

import numpy as np

import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
CLI = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "partitionedhashjoin_amd", "phjoin")


def run_cli(tmp_path, *args):
    out = tmp_path / "hashjoin.txt"
    r = subprocess.run([CLI, "--log", "debug", "-f", str(out)] + list(args), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(out.read_text()), r.stderr


@pytest.mark.parametrize("args,type_", [
    (("--join", "radix-partitioning"), "RadixParitioning"),
    (("--join", "radix-partitioning", "-p", "1024"), "RadixParitioning"),
    (("--join", "radix-partitioning", "--radix-bits", "8,8", "--hash", "murmur3"), "RadixParitioning"),
    (("--join", "no-partitioning"), "NoPartitioning"),
])
def test_cli_matches_oracle(tmp_path, args, type_):
    nR, nS, skew, seed = 200_000, 3_000_000, 1.25, 4242
    res, log = run_cli(tmp_path, "--primary", str(nR), "--secondary", str(nS), "--skew", str(skew),
                       "--seed", str(seed), "-u", "us", *args)
    R, S = O.generate_tables(nR, nS, skew, seed)      # the CLI's host generator == the oracle's
    expect = O.join_radix(R, S, P=256, workers=4).matches
    assert int(res["device"]["matches"]) == expect == nS
    assert res["id"] == "hashjointimingresult"
    assert res["parameters"]["Type"] == type_
    assert res["parameters"]["PrimaryRelationSize"] == str(nR)
    # exactly the reference's phases: generate.sh pastes every .results value as a row
    assert list(res["results"]) == ["partition", "build", "probe"]
    assert f"Joined" in log and str(expect) in log


def test_cli_device_generation(tmp_path):
    res, _ = run_cli(tmp_path, "--primary", "1000000", "--secondary", "20000000", "--generate", "device",
                     "--join", "radix-partitioning", "--radix-bits", "8,8")
    assert int(res["device"]["matches"]) == 20_000_000
    assert res["parameters"]["NumberOfPartitions"] == "65536"


def test_cli_primary_one_terminates_like_reference(tmp_path):
    # --primary 1 makes Zipf reject the [1, 1] range outside the join's try block
    # (src/main.cpp:68-74, Zipf.cpp:61-67): the process terminates abnormally
    r = subprocess.run([CLI, "--join", "radix-partitioning", "--primary", "1", "--secondary", "10",
                        "-f", str(tmp_path / "x.txt")], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "Range for Zipf generation is incorrectly specified" in r.stderr


@pytest.mark.parametrize("join", ["radix-partitioning", "no-partitioning"])
def test_cli_materialize_rows(tmp_path, join):
    # --materialize on: Run() returns one JoinedTuple per probe tuple; Sequential
    # R has unique keys, so payloadA = id - 1 and the row checksum is exact
    nR, nS, seed = 100_000, 1_500_000, 77
    res, _ = run_cli(tmp_path, "--primary", str(nR), "--secondary", str(nS), "--seed", str(seed),
                     "--join", join, "--materialize", "on")
    R, S = O.generate_tables(nR, nS, 1.05, seed)
    ids = S[:, 0].astype(np.uint64)
    want = int((ids * np.uint64(3) + (ids - np.uint64(1)) * np.uint64(5)
                + S[:, 1].astype(np.uint64) * np.uint64(7)).sum(dtype=np.uint64))
    assert int(res["device"]["rows"]) == int(res["device"]["matches"]) == nS
    assert int(res["device"]["rows_checksum"]) == want


@pytest.mark.parametrize("devs,join", [
    (("--exchange", "rccl"), "radix-partitioning"),            # RCCL world of one (phj_ctx_create_ex)
    (("--exchange", "rccl"), "no-partitioning"),
    (("--exchange", "local", "--devices", "0,0,0"), "radix-partitioning"),   # 3 ranks on one GPU
    (("--exchange", "local", "--devices", "0,0"), "no-partitioning"),
])
def test_cli_multi_device_context(tmp_path, devs, join):
    # the multi-GPU join through the reference's own entry point (phjoin ->
    # Gpu::HashJoiner::Run -> multi-device phj_ctx): same count, reference
    # JSON, plus the device object's gpus / exchange_us
    nR, nS, skew, seed = 200_000, 3_000_000, 1.05, 99
    res, log = run_cli(tmp_path, "--primary", str(nR), "--secondary", str(nS), "--skew", str(skew),
                       "--seed", str(seed), "--join", join, *devs)
    assert int(res["device"]["matches"]) == nS
    ndev = len(devs[3].split(",")) if len(devs) > 2 else 1
    assert int(res["device"]["gpus"]) == ndev
    assert "exchange_us" in res["device"]
    assert list(res["results"]) == ["partition", "build", "probe"]
