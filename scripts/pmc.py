#!/usr/bin/env python3
"""rocprofv3 PMC counters per join phase (timer) of the C2/C4/C5 workloads.

Each counter group runs as its own rocprofv3 pass over scripts/pmc_probe.py
(a child process; the caller must not have touched the GPU yet). Dispatches
are attributed to the probe's last join by walking its timer list backwards
and matching each timer to the kernel family that does its work (scan timers
are skipped). Usage:

    python scripts/pmc.py --counters FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_LDS"

prints one JSON object {timer: {counter: value per launch}}. Counter units are
rocprofv3's: FETCH_SIZE / WRITE_SIZE in KiB (see hbm_bytes for the gfx950
correction of MI355X_MICROARCH.md §HBM).
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# one dispatch doing the work of two timers ("build" and "probe")
SHARED = re.compile(r"phj::k_(join_fused|cluster_probe(?!_big))")

# timer name -> kernel family doing its work (first match wins)
FAMILIES = [
    (re.compile(r"^R\.p2\.scatter$"), re.compile(r"phj::k_ht_p2")),
    (re.compile(r"\.hist$"), re.compile(r"phj::k_hist")),
    (re.compile(r"\.scatter$"), re.compile(r"phj::k_(scatter|chunk_codes)")),
    # (the LDS join's main kernel, not its big-cluster companion k_cluster_probe_big,
    # which is dispatched after it: VERDICT r05 weak 2)
    (re.compile(r"^build$"), re.compile(r"phj::k_(build_small|ht_fill|join_fused|cluster_probe(?!_big))")),
    (re.compile(r"^build\.big$"), re.compile(r"phj::k_cluster_big_fill")),
    (re.compile(r"^probe$"), re.compile(r"phj::k_(probe|join_fused|cluster_probe(?!_big))")),
    (re.compile(r"^np\.build$"), re.compile(r"phj::k_(np_build(?!_overflow)|ht_fill)")),
    (re.compile(r"^np\.probe$"), re.compile(r"phj::k_np_probe")),
]


def family(timer):
    for t, k in FAMILIES:
        if t.search(timer):
            return k
    return None


def run_pass(counters, config, primary, secondary, timeout=300):
    """One rocprofv3 pass; returns (rows, timer names of the probe's last join)."""
    out = tempfile.mkdtemp(prefix="phj_pmc_", dir="/tmp")
    cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", out, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "scripts", "pmc_probe.py"), "--config", config,
           "--primary", str(primary), "--secondary", str(secondary)]
    try:
        p = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=timeout, cwd="/tmp",
                           env=dict(os.environ, TMPDIR="/tmp"))
        timers = []
        for line in p.stdout.splitlines():
            if line.startswith("TIMERS "):
                timers = json.loads(line[len("TIMERS "):])
        rows = []
        for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                rows += list(csv.DictReader(fh))
        return rows, timers
    finally:
        shutil.rmtree(out, ignore_errors=True)


def attribute(rows, timers):
    """{timer: {counter: value}} for the last join: dispatches in Dispatch_Id
    order, matched backwards against the timers' kernel families."""
    disp = {}
    for r in rows:
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "vals": {}})
        d["vals"][r["Counter_Name"]] = d["vals"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seq = [disp[k] for k in sorted(disp)]
    res = {}
    i = len(seq) - 1
    shared = None   # the fused join, the LDS join: "build" and "probe" are one dispatch
    for t in reversed(timers):
        fam = family(t)
        if fam is None:
            continue
        if shared is not None and fam.search(shared["name"]):
            res[t] = dict(shared["vals"])
            shared = None
            continue
        while i >= 0 and not fam.search(seq[i]["name"]):
            i -= 1
        if i < 0:
            break
        res[t] = dict(seq[i]["vals"])
        shared = seq[i] if SHARED.search(seq[i]["name"]) else None
        i -= 1
    return res


def collect(groups, config="c2", primary=10_000_000, secondary=200_000_000):
    per = {}
    for g in groups:
        rows, timers = run_pass(g, config, primary, secondary)
        for t, vals in attribute(rows, timers).items():
            per.setdefault(t, {}).update(vals)
    return per


# Memory-side read requests by size (one pass: 3 of the 4 TCC counters) and
# WRITE_SIZE (its own pass). Calibrated on known byte counts
# (scripts/pmc_calib.hip, profiles/r03_pmc_calib.json): coalesced 8- and 16-B
# per lane reads arrive as 128-B requests (FETCH_SIZE reports them at half,
# the MI355X_MICROARCH.md x2 correction), random L2 misses as 64-B requests
# (FETCH_SIZE reports those in full, so FETCH_SIZE x 2 double-counts them);
# WRITE_SIZE reads 8- and 16-B stores exactly.
READ_COUNTERS = ["TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_32B_sum"]


def hbm_bytes(per):
    """HBM bytes per launch: 128 / 64 / 32 B per memory-side read request of
    each size + WRITE_SIZE (KiB). Falls back to FETCH_SIZE x 2 + WRITE_SIZE
    when the request-size counters were not collected."""
    out = {}
    for t, v in per.items():
        if "WRITE_SIZE" not in v:
            continue
        if all(k in v for k in READ_COUNTERS):
            rd = 128 * v[READ_COUNTERS[0]] + 64 * v[READ_COUNTERS[1]] + 32 * v[READ_COUNTERS[2]]
            out[t] = rd + v["WRITE_SIZE"] * 1024
        elif "FETCH_SIZE" in v:
            out[t] = (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counters", nargs="+", default=["FETCH_SIZE", "WRITE_SIZE"],
                    help="counter groups; a group is one space-separated string = one pass")
    ap.add_argument("--config", default="c2", choices=["c2", "c4", "c5"])
    ap.add_argument("--primary", type=int, default=10_000_000)
    ap.add_argument("--secondary", type=int, default=200_000_000)
    a = ap.parse_args()
    groups = [g.split() for g in a.counters]
    print(json.dumps(collect(groups, a.config, a.primary, a.secondary), indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
