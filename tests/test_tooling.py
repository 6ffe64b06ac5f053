"""Measurement tooling that runs without a GPU: PMC dispatch attribution
(scripts/pmc.py) used by bench.py's roofline traffic."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import pmc  # noqa: E402


def _rows(names, counter="FETCH_SIZE"):
    return [{"Dispatch_Id": str(i + 1), "Kernel_Name": n, "Counter_Name": counter, "Counter_Value": str(i)}
            for i, n in enumerate(names)]


def test_attribution_takes_the_last_join_in_order():
    join = ["void phj::k_hist<512, 8, true, 1>(phj::PassArgs)", "phj::k_scan_reduce(phj::ScanArgs)",
            "void phj::k_scatter<512, 8, true, true, 1>(phj::PassArgs)", "void phj::k_hist_col<4096, unsigned char>",
            "void phj::k_scatter<512, 8, true, false, 1>(phj::PassArgs)", "phj::k_join_prep(...)",
            "void phj::k_build_small<1>(phj::BuildArgs)", "void phj::k_build_big<1>(phj::BuildArgs)",
            "void phj::k_probe<1, 8, 2>(phj::ProbeArgs)"]
    names = ["phj::k_count_range(...)"] + join + join   # two joins: the second one is reported
    timers = ["S.p1.hist", "S.p1.scan", "S.p1.scatter", "S.p2.hist", "S.p2.scan", "S.p2.scatter", "build", "probe"]
    got = pmc.attribute(_rows(names), timers)
    off = 1 + len(join)
    assert got["S.p1.hist"]["FETCH_SIZE"] == off + 0
    assert got["S.p1.scatter"]["FETCH_SIZE"] == off + 2
    assert got["S.p2.hist"]["FETCH_SIZE"] == off + 3
    assert got["S.p2.scatter"]["FETCH_SIZE"] == off + 4
    assert got["build"]["FETCH_SIZE"] == off + 6
    assert got["probe"]["FETCH_SIZE"] == off + 8
    assert "S.p1.scan" not in got


def test_hbm_bytes_gfx950_correction():
    per = {"probe": {"FETCH_SIZE": 100.0, "WRITE_SIZE": 10.0}, "build": {"FETCH_SIZE": 1.0}}
    assert pmc.hbm_bytes(per) == {"probe": (200 + 10) * 1024}
    # request-size counters (calibrated: 128-B streaming requests, 64-B random misses) win when present
    per = {"probe": {"FETCH_SIZE": 100.0, "WRITE_SIZE": 10.0, "TCC_EA0_RDREQ_128B_sum": 5.0,
                     "TCC_EA0_RDREQ_64B_sum": 3.0, "TCC_EA0_RDREQ_32B_sum": 1.0}}
    assert pmc.hbm_bytes(per) == {"probe": 5 * 128 + 3 * 64 + 32 + 10 * 1024}


def test_every_tuning_knob_has_a_schedule_test():
    # every PHJ_* variable the library reads selects a schedule that
    # tests/test_gpu_schedules.py runs (PHJ_REHEARSE: tests/test_gpu_multirank.py)
    import glob
    import re
    src = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "partitionedhashjoin_amd", "csrc", "*")))
    knobs = set(re.findall(r'(?:env_int|getenv)\("(PHJ_[A-Z0-9_]+)"', src))
    tested = open(os.path.join(ROOT, "tests", "test_gpu_schedules.py")).read() + \
        open(os.path.join(ROOT, "tests", "test_gpu_multirank.py")).read()
    assert knobs, "no knobs found"
    missing = sorted(k for k in knobs if f'"{k}"' not in tested)
    assert not missing, missing


def test_fused_join_is_one_dispatch_for_build_and_probe():
    join = ["void phj::k_hist<512, 8, true, 1>(phj::PassArgs)", "void phj::k_scatter<512, 8, true, true, 1>",
            "phj::k_fused_items(...)", "void phj::k_join_fused<1, 4, 512>(phj::FusedArgs)"]
    names = join + join
    timers = ["S.p1.hist", "S.p1.scatter", "build", "probe"]
    got = pmc.attribute(_rows(names), timers)
    assert got["build"] == got["probe"] == {"FETCH_SIZE": 7.0}
    assert got["S.p1.scatter"]["FETCH_SIZE"] == 5
    assert got["S.p1.hist"]["FETCH_SIZE"] == 4


def test_lds_join_traffic_is_the_main_kernel_not_its_big_companion():
    """`build` / `probe` took k_cluster_probe_big's
    counters (a 7.9 us launch dispatched after the LDS join) instead of
    k_cluster_probe's."""
    join = ["void phj::k_chunk_codes_pipe<1024, 4, 1, 1, 0, false, 2>(phj::PassArgs, unsigned int, unsigned int)",
            "phj::k_pass1_finish_sizes(...)", "phj::k_tile_chunks(...)",
            "void phj::k_chunk_codes_pipe<1024, 4, 1, 1, 0, false, 1>(phj::PassArgs, unsigned int, unsigned int)",
            "phj::k_pass1_finish_sizes(...)", "phj::k_tile_chunks(...)",
            "phj::k_cluster_big_fill(phj::ClusterArgs)",
            "void phj::k_cluster_probe<1024, 4, 3, true, false, true, true>(phj::ClusterArgs)",
            "phj::k_cluster_probe_big(phj::ClusterArgs)"]
    names = join + join
    timers = ["S.p1.scatter", "R.p1.scatter", "build.big", "build", "probe"]   # (pmc_probe.py: every timer)
    got = pmc.attribute(_rows(names), timers)
    off = len(join)
    assert got["build"] == got["probe"] == {"FETCH_SIZE": float(off + 7)}
    assert got["build.big"]["FETCH_SIZE"] == off + 6
    assert got["R.p1.scatter"]["FETCH_SIZE"] == off + 3
    assert got["S.p1.scatter"]["FETCH_SIZE"] == off + 0


def test_sweep_writes_generate_sh_figure_layout(tmp_path):
    # scripts/sweep.py writes the reference's figure.dat layout (generate.sh:66-82):
    # one column per run, rows NumberOfPartitions / Partition / Build / Probe
    import sweep
    names = [n for n, _a, _p in sweep.columns()]
    assert names[0] == "NoPartitioning" and names[1:] == [f"Radix{p}" for p in sweep.PARTITIONS]
    table = {n: {"partition": i, "build": 2 * i, "probe": 3 * i} for i, n in enumerate(names)}
    path = tmp_path / "fig.dat"
    sweep.write_figure(str(path), table)
    rows = [line.split() for line in path.read_text().splitlines()]
    assert [r[0] for r in rows] == ["NumberOfPartitions", "Partition", "Build", "Probe"]
    assert rows[0][1:] == names
    assert rows[3][1:] == [str(3 * i) for i in range(len(names))]
