#!/usr/bin/env python3
"""PMC counters of the last dispatch of the kernels matching a regex, over
env-variant runs of scripts/pmc_probe.py (one rocprofv3 --pmc pass per
counter group, each a child process; run from a process that has not touched
the GPU). Prints one JSON line per variant: {kernel: {counter: value}}.

  python scripts/pmc_kernel.py --config c4 --kernel np_probe \
      --group TCC_HIT_sum,TCC_MISS_sum --variant PHJ_P1_WPC2=2 --variant PHJ_P1_WPC2=4
"""
import argparse
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--kernel", required=True, help="regex over kernel names")
    ap.add_argument("--group", action="append", required=True, help="comma-separated counters of one pass")
    ap.add_argument("--variant", action="append", default=[], help="VAR=VAL[,VAR=VAL] environment of a run")
    ap.add_argument("--primary", type=int, default=10_000_000)
    ap.add_argument("--secondary", type=int, default=200_000_000)
    a = ap.parse_args()
    rx = re.compile(a.kernel)
    for var in a.variant or [""]:
        env = dict(kv.split("=", 1) for kv in var.split(",") if kv)
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        out = {}
        try:
            for g in a.group:
                rows, _ = pmc.run_pass(g.split(","), a.config, a.primary, a.secondary, timeout=120)
                last = {}
                for r in rows:
                    if rx.search(r["Kernel_Name"]):
                        d = int(r["Dispatch_Id"])
                        last.setdefault(d, {"name": r["Kernel_Name"][:60], "vals": {}})
                        v = last[d]["vals"]
                        v[r["Counter_Name"]] = v.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                if last:
                    d = last[max(last)]
                    out.setdefault(d["name"], {}).update(d["vals"])
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        print(json.dumps({"variant": var, "counters": out}), flush=True)


if __name__ == "__main__":
    main()
