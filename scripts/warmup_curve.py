#!/usr/bin/env python3
"""Per-block step times of the C2 join from a process's first GPU work on:
how long a fresh box runs slower (clock / power state) before its steady rate.
Prints one JSON line per block of --block steps."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=30)
    ap.add_argument("--block", type=int, default=50)
    a = ap.parse_args()
    import partitionedhashjoin_amd as phj
    t_start = time.perf_counter()
    c = phj.Context(0)
    c.generate_sequential(0, 10_000_000, 1)
    c.generate_zipf(1, 200_000_000, 1.05, 1, 10_000_000, 20240601)
    p = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3)
    c.prepare(p)
    q = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3)
    q.flags |= phj.DEFER_TIMERS | phj.LEAN_TIMERS
    c.timers_report()
    for b in range(a.blocks):
        t0 = time.perf_counter()
        for _ in range(a.block):
            c.join(q)
        c.synchronize()
        dt = (time.perf_counter() - t0) * 1e3 / a.block
        rep = {n: round(ms / a.block, 4) for n, ms, _ in c.timers_report().timers() if n in ("S.p1.scatter", "probe", "build")}
        print(json.dumps({"block": b, "since_start_s": round(time.perf_counter() - t_start, 2), "ms_per_step": round(dt, 4),
                          **rep}), flush=True)


if __name__ == "__main__":
    main()
