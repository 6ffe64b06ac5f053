#!/usr/bin/env python3
"""Per-rank device work of the N-GPU C2 step, rehearsed on one GPU.

A PHJ_CTX_LOCAL context with W members on device 0 runs the multi-GPU member
step of csrc/phj_group.h (R shard partition + pack, the exchange as device
copies, the probe side's pass 1 and the on-chip pass 2 + probe against the W
gathered build segments). With PHJ_REHEARSE=1 members 1..W-1 only partition
and pack their R shards (what the all-gather delivers) and member 0 runs the
whole step, so member 0's time is one rank's device work at world size W
(the RCCL transfer itself, 80 MB of keys in total over xGMI, is replaced by
device copies). Prints one JSON line per W.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lean-timers", action="store_true",
                    help="PHJ_LEAN_TIMERS (measured 0.008 ms slower at W=8: profiles/r05zi_ab_member_marks.txt)")
    ap.add_argument("--primary", type=int, default=10_000_000)
    ap.add_argument("--secondary", type=int, default=200_000_000)
    a = ap.parse_args()
    os.environ["PHJ_REHEARSE"] = "1"
    import partitionedhashjoin_amd as phj
    from partitionedhashjoin_amd import shard_range
    p = phj.radix_params((8, 8))
    if a.lean_timers:
        p.flags |= phj.LEAN_TIMERS
    nR, nS = a.primary, a.secondary
    for W in a.worlds:
        with phj.Context(devices=[0] * W, flags=phj.CTX_LOCAL) as g:
            g.generate_sequential(0, nR, 1)
            g.generate_zipf(1, nS, 1.05, 1, nR, 20240601)
            lo, hi = shard_range(nS, 0, W)
            g.prepare(p)
            for _ in range(3):
                r = g.join(p)
            acc, tot = {}, 0.0
            t0 = time.perf_counter()
            for _ in range(a.steps):
                r = g.join(p)
                tot += r.total_ms
                for name, ms, _b in r.timers():
                    acc[name] = acc.get(name, 0.0) + ms
            wall = (time.perf_counter() - t0) * 1e3 / a.steps
        print(json.dumps({"world": W, "rank0_device_ms": round(tot / a.steps, 4), "wall_ms_all_members": round(wall, 4),
                          "matches_rank0": int(r.matches), "s_shard": hi - lo,
                          "kernels_ms": {k: round(v / a.steps, 4) for k, v in sorted(acc.items())}}), flush=True)


if __name__ == "__main__":
    main()
