#!/usr/bin/env python3
"""Per-rank device work of the N-GPU C2 step, rehearsed on one GPU.

At world size W each rank partitions its R shard (|R|/W) and its S shard
(|S|/W), packs the partitioned R shard for the all-gather, then builds over
the W gathered R shards and probes its S shard. This script times exactly
that sequence on one GPU, with the other ranks' partitioned R shards
prepared beforehand by separate contexts (what the all-gather delivers). The
RCCL transfer itself (|R| x 16 B in total, overlapped with the S partition)
is not included. Prints one JSON line per W.
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
    ap.add_argument("--primary", type=int, default=10_000_000)
    ap.add_argument("--secondary", type=int, default=200_000_000)
    a = ap.parse_args()
    import torch
    import partitionedhashjoin_amd as phj
    from partitionedhashjoin_amd.distributed import HipShardEngine, max_shard, shard_range
    p = phj.radix_params((8, 8))
    nR, nS = a.primary, a.secondary
    for W in a.worlds:
        eng = HipShardEngine(0)
        others = []
        segs = []
        for g in range(1, W):   # the other ranks' partitioned R shards
            c = phj.Context(0)
            lo, hi = shard_range(nR, g, W)
            c.generate_sequential(0, hi - lo, 1, lo)
            segs.append(c.partition(0, p))
            c.synchronize()
            others.append(c)
        eng.generate(nR, nS, 1.05, 20240601, 0, W)
        torch.cuda.synchronize()
        maxn = max_shard(nR, W)

        def step():   # the issue order of distributed_join
            if W == 1:
                eng.partition(1, p)
                v = eng.partition(0, p)
            else:
                fut = eng.partition_async(1, p)
                v = eng.partition(0, p)
                eng.pack(v, maxn, v.num_partitions)
                fut.result()
            eng.build_ready()
            cnt = eng._count()
            eng.ctx.join_partitioned_async(p, [v] + segs, cnt.data_ptr())
            return int(cnt.item())

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        eng.timers()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            m = step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.steps
        acc = {name: v / a.steps for name, v, _ in eng.timers()}
        lo, hi = shard_range(nS, 0, W)
        print(json.dumps({"world": W, "ms_per_step": round(ms, 4), "matches_rank0": m, "s_shard": hi - lo,
                          "kernels_ms": {k: round(v, 4) for k, v in acc.items()},
                          "kernel_sum_ms": round(sum(acc.values()), 4)}), flush=True)
        for c in others:
            c.close()
        eng.ctx.close()
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
