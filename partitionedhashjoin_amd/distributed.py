"""Multi-GPU radix join: one process per GPU, torch.distributed (RCCL over xGMI).

The reference is single-process (no distributed runtime), so
this layer is new and follows BASELINE.json's north star: both relations
are range-sharded across the ranks; every rank radix-partitions its R and S
shards; the partitioned build shards are exchanged with one all-gather (the
only data-path collective: S, 95% of the bytes, never leaves its GPU and
stays balanced under any key skew); each rank joins its S shard against the
gathered build side partition by partition; the counts are summed with an
all-reduce.

The exchange overlaps the S-side partitioning: the all-gather is issued
asynchronously after the R partition, S is partitioned on the compute
stream meanwhile, and the join waits on the collective.

`ShardEngine` is the per-rank compute interface. `HipShardEngine` drives
libphj_hip.so on the rank's GPU; tests substitute a CPU engine to exercise
this orchestration with the gloo backend.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def shard_range(n: int, rank: int, world: int):
    """Rows [lo, hi) of an n-row relation owned by `rank` (contiguous range shard)."""
    lo = (n * rank) // world
    hi = (n * (rank + 1)) // world
    return lo, hi


def max_shard(n: int, world: int) -> int:
    return max(hi - lo for lo, hi in (shard_range(n, r, world) for r in range(world)))


@dataclass
class DistResult:
    matches: int             # global semi-join count (all-reduced)
    local_matches: int
    build_ms: float          # this rank's device phases (hipEvents)
    probe_ms: float
    timers: list


class HipShardEngine:
    """Per-rank engine over libphj_hip.so; tensors live on the rank's GPU."""

    def __init__(self, device: int):
        import torch
        from . import Context
        self.torch = torch
        self.device = torch.device("cuda", device)
        torch.cuda.set_device(self.device)
        self.ctx = Context(device)
        # run every kernel on torch's current stream so RCCL collectives order after them
        self.ctx.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def tensor(self, n, dtype):
        return self.torch.empty(int(n), dtype=dtype, device=self.device)

    def generate(self, nR, nS, alpha, seed, rank, world):
        rlo, rhi = shard_range(nR, rank, world)
        slo, shi = shard_range(nS, rank, world)
        self.ctx.generate_sequential(0, rhi - rlo, 1, rlo)
        self.ctx.generate_zipf(1, shi - slo, alpha, 1, nR, seed, slo)

    def partition(self, side, params):
        return self.ctx.partition(side, params)

    def export(self, view, maxn):
        """Copy a partitioned build view into fixed-size tensors for the all-gather."""
        import ctypes as C
        torch = self.torch
        keys = self.tensor(maxn, torch.int64)
        pays = self.tensor(maxn, torch.int64)
        bounds = self.tensor(view.num_partitions + 1, torch.int32)
        L = self.ctx._L
        self.ctx._check(L.phj_partitioned_download(self.ctx._h, C.byref(view),
                                                   C.c_void_p(keys.data_ptr()),
                                                   C.c_void_p(pays.data_ptr()),
                                                   C.c_void_p(bounds.data_ptr())))
        return keys, pays, bounds

    def join_gathered(self, params, keys_all, pays_all, bounds_all, sizes, maxn, P):
        from ._capi import Partitioned
        segs = []
        for g, n in enumerate(sizes):
            v = Partitioned()
            v.keys = keys_all.data_ptr() + g * maxn * 8
            v.payloads = pays_all.data_ptr() + g * maxn * 8
            v.bounds = bounds_all.data_ptr() + g * (P + 1) * 4
            v.n = n
            v.num_partitions = P
            segs.append(v)
        return self.ctx.join_partitioned(params, segs)

    def join_local(self, params, view):
        return self.ctx.join_partitioned(params, [view])

    def count_tensor(self, value):
        return self.torch.tensor([value], dtype=self.torch.int64, device=self.device)


def _all_gather(dist, out, inp):
    """all_gather_into_tensor; device tensors are staged through host memory
    when the process group is gloo (CPU-only collectives: rehearsal runs)."""
    if inp.is_cuda and dist.get_backend() == "gloo":
        host_out = out.new_empty(out.shape, device="cpu")
        dist.all_gather_into_tensor(host_out, inp.cpu())
        out.copy_(host_out)
        return None
    return dist.all_gather_into_tensor(out, inp, async_op=True)


def _all_reduce(dist, t):
    if t.is_cuda and dist.get_backend() == "gloo":
        h = t.cpu()
        dist.all_reduce(h)
        t.copy_(h)
    else:
        dist.all_reduce(t)


def distributed_join(engine, params, nR: int, nS: int, rank: int, world: int, dist=None):
    """Join the range-sharded relations already resident on every rank.

    engine.partition(side) partitions this rank's shard (R side 0, S side 1).
    With world == 1 no collective runs.
    """
    torch = engine.torch
    view = engine.partition(0, params)
    P = view.num_partitions
    maxn = max_shard(nR, world)
    sizes = [hi - lo for lo, hi in (shard_range(nR, r, world) for r in range(world))]
    if world > 1:
        keys, pays, bounds = engine.export(view, maxn)
        keys_all = engine.tensor(world * maxn, torch.int64)
        pays_all = engine.tensor(world * maxn, torch.int64)
        bounds_all = engine.tensor(world * (P + 1), torch.int32)
        works = [_all_gather(dist, keys_all, keys), _all_gather(dist, pays_all, pays),
                 _all_gather(dist, bounds_all, bounds)]
        engine.partition(1, params)         # overlaps the exchange
        for w in works:
            if w is not None:
                w.wait()
        res = engine.join_gathered(params, keys_all, pays_all, bounds_all, sizes, maxn, P)
        cnt = engine.count_tensor(res.matches)
        _all_reduce(dist, cnt)
        total = int(cnt.item())
    else:
        engine.partition(1, params)
        res = engine.join_local(params, view)
        total = int(res.matches)
    timers = res.timers() if hasattr(res, "timers") else []
    return DistResult(matches=total, local_matches=int(res.matches),
                      build_ms=float(getattr(res, "build_ms", 0.0)),
                      probe_ms=float(getattr(res, "probe_ms", 0.0)), timers=timers)


def gathered_segments_numpy(keys_all, pays_all, bounds_all, sizes, maxn, P):
    """Split gathered buffers back into per-rank (keys, payloads, bounds) numpy views."""
    keys_all = np.asarray(keys_all)
    pays_all = np.asarray(pays_all)
    bounds_all = np.asarray(bounds_all).astype(np.int64) & 0xFFFFFFFF
    segs = []
    for g, n in enumerate(sizes):
        segs.append((keys_all[g * maxn:g * maxn + n], pays_all[g * maxn:g * maxn + n],
                     bounds_all[g * (P + 1):(g + 1) * (P + 1)]))
    return segs
