#!/usr/bin/env python3
"""GPU equivalent of the reference's scripts/generate.sh sweep.

Runs the phjoin CLI for NoPartitioning and RadixCluster with
P in {32, ..., 8192} at each requested skew and writes, per skew, the
reference's figure.dat layout (rows NumberOfPartitions / Partition / Build /
Probe, one column per run; generate.sh:66-82) plus a JSON file with the
device-side extras. Unlike generate.sh:78, the radix runs use the requested
skew (the reference script hard-codes 1.05 there).

    python scripts/sweep.py --skew 1.05 1.25 --out profiles/r01_sweep_cli
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


def run(args, unit):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.txt")
        cmd = [CLI, *args, "-u", unit, "--log", "error", "-o", "file", "--filename", out]
        subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=600)
        with open(out) as f:
            return json.load(f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skew", type=float, nargs="+", default=[1.05, 1.25])
    ap.add_argument("--primary", type=int, default=10_000_000)
    ap.add_argument("--secondary", type=int, default=200_000_000)
    ap.add_argument("--unit", default="us")
    ap.add_argument("--generate", default="device", choices=["host", "device"])
    ap.add_argument("--out", default="sweep")
    a = ap.parse_args()
    common = ["--primary", str(a.primary), "--secondary", str(a.secondary), "--generate", a.generate]
    for skew in a.skew:
        cols = [("NoPartitioning", ["--join", "no-partitioning"])]
        cols += [(f"Radix{p}", ["--join", "radix-partitioning", "-p", str(p)]) for p in PARTITIONS]
        table = {}
        for name, args in cols:
            res = run(args + common + ["--skew", str(skew)], a.unit)
            r = res["results"]
            table[name] = {"partition": int(r["partition"]), "build": int(r["build"]), "probe": int(r["probe"]),
                           **{k: v for k, v in res.get("device", {}).items()}}
            print(f"skew {skew} {name:16s} {r['partition']:>8s} {r['build']:>8s} {r['probe']:>8s} "
                  f"matches {res.get('device', {}).get('matches')}", flush=True)
        rows = [["NumberOfPartitions"] + list(table), ["Partition"] + [str(v["partition"]) for v in table.values()],
                ["Build"] + [str(v["build"]) for v in table.values()],
                ["Probe"] + [str(v["probe"]) for v in table.values()]]
        base = f"{a.out}_{skew}"
        with open(base + ".dat", "w") as f:
            f.write("\n".join(" ".join(r) for r in rows) + "\n")
        with open(base + ".json", "w") as f:
            json.dump({"skew": skew, "unit": a.unit, "primary": a.primary, "secondary": a.secondary,
                       "runs": table}, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
