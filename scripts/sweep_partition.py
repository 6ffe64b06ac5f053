#!/usr/bin/env python3
"""Launch-shape sweep for the partition passes (GPU; results are launch-shape
independent, so only time is compared). Prints one JSON object per variant.

  python scripts/sweep_partition.py [--reps 5] [--mode join|bits]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def avg_timers(results):
    acc = {}
    for r in results:
        for name, ms, nbytes in r.timers():
            a = acc.setdefault(name, [0.0, 0])
            a[0] += ms
            a[1] = nbytes
    return {k: (v[0] / len(results), v[1]) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--mode", default="join")
    ap.add_argument("--nR", type=int, default=10_000_000)
    ap.add_argument("--nS", type=int, default=200_000_000)
    ap.add_argument("--alpha", type=float, default=1.05)
    ap.add_argument("--variants", default="", help="JSON list of env dicts (join mode)")
    args = ap.parse_args()
    import partitionedhashjoin_amd as phj

    import torch
    x = torch.empty(args.nS * 2, dtype=torch.int64, device="cuda")
    y = torch.empty_like(x)
    x.fill_(1)
    for _ in range(3):
        y.copy_(x)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(10):
        y.copy_(x)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / 10
    print(json.dumps({"torch_copy_ms": ms, "GBps": 2 * x.numel() * 8 / ms / 1e6}), flush=True)
    del x, y
    torch.cuda.empty_cache()

    base = phj.Context(0)
    base.generate_sequential(0, args.nR, 1)
    base.generate_zipf(1, args.nS, args.alpha, 1, args.nR, 20240601)
    rptr, nR = base.relation_ptr(0)
    sptr, nS = base.relation_ptr(1)

    def make_ctx(env):
        for k in list(os.environ):
            if k.startswith("PHJ_"):
                os.environ.pop(k, None)
        os.environ.update({k: str(v) for k, v in env.items()})
        c = phj.Context(0)
        c.bind_device(0, rptr, nR)
        c.bind_device(1, sptr, nS)
        return c

    if args.mode == "join":
        if args.variants:
            variants = json.loads(args.variants)
        else:
            variants = []
            for items in (8, 16):
                for aos in (0, 1):
                    for remap in (0, 1):
                        variants.append({"PHJ_WC": 0, "PHJ_TILE_ITEMS": items, "PHJ_P1_AOS": aos,
                                         "PHJ_XCD_REMAP": remap})
        for env in variants:
            c = make_ctx(env)
            p = phj.radix_params((8, 8))
            c.join(p)
            rs = [c.join(p) for _ in range(args.reps)]
            t = avg_timers(rs)
            out = {"variant": env, "total_ms": sum(r.total_ms for r in rs) / len(rs),
                   "matches": rs[-1].matches,
                   "kernels": {k: [round(v[0], 4), round(v[1] / v[0] / 1e6, 1)] for k, v in t.items()}}
            print(json.dumps(out), flush=True)
            c.close()
    else:
        for env in ({}, {"PHJ_TILE_ITEMS": 16}, {"PHJ_XCD_REMAP": 1}):
            c = make_ctx(env)
            for bits in (4, 5, 6, 7, 8, 9, 10, 11):
                p = phj.radix_params((bits, 0))
                c.partition(1, p)
                c.timers_report()
                rs = []
                for _ in range(args.reps):
                    c.partition(1, p)
                    rs.append(c.timers_report())
                t = avg_timers(rs)
                print(json.dumps({"variant": env, "bits": bits,
                                  "kernels": {k: [round(v[0], 4), round(v[1] / v[0] / 1e6, 1)]
                                              for k, v in t.items()}}), flush=True)
            c.close()


if __name__ == "__main__":
    main()
