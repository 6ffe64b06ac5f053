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


class HipShardEngine:
    """One rank's work issued the way the member step of csrc/phj_group.h
    issues it: R partition + pack on a second context/stream beside the S
    partition on the main one (measurement helper)."""

    def __init__(self, device):
        import torch
        import partitionedhashjoin_amd as phj
        from concurrent.futures import ThreadPoolExecutor
        self.torch = torch
        self.device = torch.device("cuda", device)
        torch.cuda.set_device(self.device)
        self.ctx = phj.Context(device)
        self.stream = torch.cuda.Stream(self.device)
        torch.cuda.set_stream(self.stream)
        self.ctx.set_stream(self.stream.cuda_stream)
        self.ctx_r = phj.Context(device)
        self.stream_r = torch.cuda.Stream(self.device)
        self.ctx_r.set_stream(self.stream_r.cuda_stream)
        self.issuer = ThreadPoolExecutor(max_workers=1)

    def generate(self, nR, nS, alpha, seed, rank, world):
        from partitionedhashjoin_amd.distributed import shard_range
        rlo, rhi = shard_range(nR, rank, world)
        slo, shi = shard_range(nS, rank, world)
        self.ctx_r.generate_sequential(0, rhi - rlo, 1, rlo)
        self.ctx.generate_zipf(1, shi - slo, alpha, 1, nR, seed, slo)

    def partition(self, side, params):
        return (self.ctx_r if side == 0 else self.ctx).partition(side, params)

    def partition_async(self, side, params):
        return self.issuer.submit(self.partition, side, params)

    def build_ready(self):
        ev = self.torch.cuda.Event()
        ev.record(self.stream_r)
        self.stream.wait_event(ev)

    def pack(self, view, maxn, P):
        import ctypes as C
        from partitionedhashjoin_amd.distributed import pack_layout
        maxn, E = pack_layout(maxn, P)
        with self.torch.cuda.stream(self.stream_r):
            send = self.torch.empty(E, dtype=self.torch.int64, device=self.device)
        base = send.data_ptr()
        L = self.ctx_r._L
        self.ctx_r._check(L.phj_partitioned_download(self.ctx_r._h, C.byref(view), C.c_void_p(base),
                                                     C.c_void_p(0), C.c_void_p(base + maxn * 8)))
        return send

    def _count(self):
        return self.torch.zeros(1, dtype=self.torch.int64, device=self.device)

    def timers(self):
        t = {}
        for ctx in (self.ctx_r, self.ctx):
            for name, ms, nbytes in ctx.timers_report().timers():
                a = t.setdefault(name, [0.0, 0])
                a[0] += ms
                a[1] += nbytes
        return [(k, v[0], v[1]) for k, v in t.items()]



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--primary", type=int, default=10_000_000)
    ap.add_argument("--secondary", type=int, default=200_000_000)
    a = ap.parse_args()
    import torch
    import partitionedhashjoin_amd as phj
    from partitionedhashjoin_amd.distributed import max_shard, shard_range
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
        eng.ctx_r.close()
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
