#!/usr/bin/env python3
"""GPU equivalent of the reference's scripts/generate.sh sweep.

Runs the phjoin CLI for NoPartitioning and RadixCluster with
P in {32, ..., 8192} at each requested skew and GPU count, and writes, per
(skew, GPU count), the reference's figure.dat layout (rows NumberOfPartitions
/ Partition / Build / Probe, one column per run; generate.sh:66-82) plus a
JSON file with the device-side extras. Unlike generate.sh:78, the radix runs
use the requested skew (the reference script hard-codes 1.05 there).

With --cpu, the same columns are also timed on this host's cores with the
oracle's restatement of the reference's CPU path (test infrastructure, as
bench.py's cpu_baseline) over the same relations (the host generator equals
the CLI's, generate.sh's default relations), into <out>_<skew>_cpu.dat.

    python scripts/sweep.py --skew 1.05 1.25 --gpus 1 --cpu --out profiles/r02_sweep_cli

With --rehearse-worlds W..., the GPU-count axis is also REHEARSED ON ONE GPU
(for boxes with one MI355X): the CLI's multi-device step with W members on
device 0 (--devices 0,..,0 --exchange local) and PHJ_REHEARSE=1, so members
1..W-1 only feed the exchange (device copies standing in for the RCCL
all-gather) and the reported phases are member 0's, i.e. one rank's device
work at world size W (the radix columns; the NoPartitioning step has no
rehearsal form). Written to <out>_<skew>_rehearsed_w<W>.dat and one
<out>_<skew>_gpu_axis.json (per column: the total per W, labelled).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "partitionedhashjoin_amd", "phjoin")
PARTITIONS = [32, 64, 128, 256, 512, 1024, 2048, 4096, 8192]
UNIT_NS = {"ns": 1, "us": 1e3, "ms": 1e6, "s": 1e9}


def columns():
    cols = [("NoPartitioning", ["--join", "no-partitioning"], None)]
    cols += [(f"Radix{p}", ["--join", "radix-partitioning", "-p", str(p)], p) for p in PARTITIONS]
    return cols


def figure_rows(table):
    """generate.sh's figure.dat: one column per run, rows NumberOfPartitions / Partition / Build / Probe."""
    return [["NumberOfPartitions"] + list(table),
            ["Partition"] + [str(v["partition"]) for v in table.values()],
            ["Build"] + [str(v["build"]) for v in table.values()],
            ["Probe"] + [str(v["probe"]) for v in table.values()]]


def write_figure(path, table):
    with open(path, "w") as f:
        f.write("\n".join(" ".join(r) for r in figure_rows(table)) + "\n")


def run(args, unit, env=None):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.txt")
        cmd = [CLI, *args, "-u", unit, "--log", "error", "-o", "file", "--filename", out]
        subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=600,
                       env=None if env is None else dict(os.environ, **env))
        with open(out) as f:
            return json.load(f)


def cpu_table(nR, nS, skew, seed, unit, threads):
    """The reference's phases on the host (oracle restatement): radix
    partition / build (slowest worker) / probe, NoPartitioning probe from the
    build start (Results.hpp:202)."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    R, S = O.generate_tables(nR, nS, skew, seed, threads=threads)
    scale = 1e6 / UNIT_NS[unit]   # ms -> unit
    table = {}
    for name, _args, P in columns():
        if P is None:
            r = O.join_nopart(R, S, hash_kind=O.HASH_XXH3, seed=2, workers=threads)
        else:
            r = O.join_radix(R, S, P=P, workers=threads)
        table[name] = {"partition": int(round(r.partition_ms * scale)), "build": int(round(r.build_ms * scale)),
                       "probe": int(round(r.probe_ms * scale)), "matches": int(r.matches),
                       "wall": int(round(r.wall_ms * scale))}
        print(f"cpu skew {skew} {name:16s} {table[name]}", flush=True)
    return table


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skew", type=float, nargs="+", default=[1.05, 1.25])
    ap.add_argument("--gpus", type=int, nargs="+", default=[1], help="GPU counts (phjoin --gpus N)")
    ap.add_argument("--primary", type=int, default=10_000_000)
    ap.add_argument("--secondary", type=int, default=200_000_000)
    ap.add_argument("--unit", default="us")
    ap.add_argument("--generate", default="device", choices=["host", "device"])
    ap.add_argument("--seed", type=int, default=20240601)
    ap.add_argument("--cpu", action="store_true", help="also time the CPU columns (oracle restatement)")
    ap.add_argument("--cpu-threads", type=int, default=15)
    ap.add_argument("--rehearse-worlds", type=int, nargs="*", default=[],
                    help="GPU-count axis rehearsed on one GPU (W members on device 0, PHJ_REHEARSE=1)")
    ap.add_argument("--out", default="sweep")
    a = ap.parse_args()
    common = ["--primary", str(a.primary), "--secondary", str(a.secondary), "--generate", a.generate,
              "--seed", str(a.seed)]
    for skew in a.skew:
        for g in a.gpus:
            table = {}
            for name, args, _p in columns():
                res = run(args + common + ["--skew", str(skew), "--gpus", str(g)], a.unit)
                r = res["results"]
                table[name] = {"partition": int(r["partition"]), "build": int(r["build"]),
                               "probe": int(r["probe"]), **{k: v for k, v in res.get("device", {}).items()}}
                print(f"skew {skew} gpus {g} {name:16s} {r['partition']:>8s} {r['build']:>8s} {r['probe']:>8s} "
                      f"matches {res.get('device', {}).get('matches')}", flush=True)
            base = f"{a.out}_{skew}" + ("" if g == 1 else f"_gpus{g}")
            write_figure(base + ".dat", table)
            with open(base + ".json", "w") as f:
                json.dump({"skew": skew, "gpus": g, "unit": a.unit, "primary": a.primary, "secondary": a.secondary,
                           "runs": table}, f, indent=1)
        if a.rehearse_worlds:
            axis = {}
            for W in a.rehearse_worlds:
                table = {}
                for name, args, _p in columns():
                    if _p is None:   # (PHJ_REHEARSE quiets the radix member step only)
                        continue
                    res = run(args + common + ["--skew", str(skew), "--devices", ",".join(["0"] * W),
                                               "--exchange", "local"], a.unit, env={"PHJ_REHEARSE": "1"})
                    r = res["results"]
                    table[name] = {"partition": int(r["partition"]), "build": int(r["build"]),
                                   "probe": int(r["probe"]), **{k: v for k, v in res.get("device", {}).items()}}
                    axis.setdefault(name, {})[W] = table[name].get("device_total_us",
                                                                   table[name]["partition"] + table[name]["build"] +
                                                                   table[name]["probe"])
                    print(f"skew {skew} rehearsed W={W} {name:16s} {r['partition']:>8s} {r['build']:>8s} "
                          f"{r['probe']:>8s}", flush=True)
                write_figure(f"{a.out}_{skew}_rehearsed_w{W}.dat", table)
            with open(f"{a.out}_{skew}_gpu_axis.json", "w") as f:
                json.dump({"skew": skew, "unit": a.unit, "primary": a.primary, "secondary": a.secondary,
                           "label": "rehearsed on one GPU: W members on device 0 (PHJ_REHEARSE=1), member 0's "
                                    "device time = one rank's work at world size W; the exchange is device "
                                    "copies, not RCCL over xGMI",
                           "total_by_world": axis}, f, indent=1)
        if a.cpu:
            table = cpu_table(a.primary, a.secondary, skew, a.seed, a.unit, a.cpu_threads)
            write_figure(f"{a.out}_{skew}_cpu.dat", table)
            with open(f"{a.out}_{skew}_cpu.json", "w") as f:
                json.dump({"skew": skew, "unit": a.unit, "threads": a.cpu_threads, "kind": "port",
                           "primary": a.primary, "secondary": a.secondary, "runs": table}, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
