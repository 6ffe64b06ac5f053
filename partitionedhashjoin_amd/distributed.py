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

import os

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
    timers: list             # this rank's per-kernel device timers (name, ms, bytes)


def pack_layout(maxn: int, P: int):
    """int64 elements of one rank's packed build shard: keys[maxn] | bounds[P+1]
    (uint32, two per element). Only the keys travel: the join tests key
    equality and never reads a build payload (the reference's Join() only
    checks Get() for null, RadixCluster/HashJoin.hpp:295-301), which halves the
    all-gather. maxn is padded to 64 elements so every column stays 16-B
    aligned inside the gathered buffer."""
    maxn = (maxn + 63) // 64 * 64
    return maxn, maxn + (P + 2) // 2


class HipShardEngine:
    """Per-rank engine over libphj_hip.so; tensors live on the rank's GPU and
    every kernel runs on torch's current stream, so the RCCL collectives and
    the joins are ordered without host synchronization."""

    def __init__(self, device: int):
        import torch
        from . import Context
        self.torch = torch
        self.device = torch.device("cuda", device)
        torch.cuda.set_device(self.device)
        # S (probe side, the join) on the main stream, shared with torch
        # (allocations, RCCL's stream dependency); R (build side) partitions on
        # its own context and stream, concurrently with S. torch's legacy default
        # stream is handle 0, which the C ABI takes as "create an own stream",
        # so explicit streams are used.
        self.ctx = Context(device)
        self.stream = torch.cuda.Stream(self.device)
        torch.cuda.set_stream(self.stream)
        self.ctx.set_stream(self.stream.cuda_stream)
        self.ctx_r = Context(device)
        self.stream_r = torch.cuda.Stream(self.device)
        self.ctx_r.set_stream(self.stream_r.cuda_stream)
        # a second host thread issues the S partition while the main thread issues
        # R, the pack and the all-gather (ctypes releases the GIL; the two contexts
        # and streams are independent)
        from concurrent.futures import ThreadPoolExecutor
        self.issuer = ThreadPoolExecutor(max_workers=1, thread_name_prefix="phj-s-issue")

    def partition_async(self, side, params):
        """Issue a partition from the issuer thread; returns a future of the view."""
        return self.issuer.submit(self.partition, side, params)

    def tensor(self, n, dtype):
        return self.torch.empty(int(n), dtype=dtype, device=self.device)

    def generate(self, nR, nS, alpha, seed, rank, world):
        rlo, rhi = shard_range(nR, rank, world)
        slo, shi = shard_range(nS, rank, world)
        self.ctx_r.generate_sequential(0, rhi - rlo, 1, rlo)
        self.ctx.generate_zipf(1, shi - slo, alpha, 1, nR, seed, slo)
        self.share_build()

    def share_build(self):
        """Make the main context see the R shard owned by the R context (for
        single-call joins such as NoPartitioning on the main context)."""
        ptr, n = self.ctx_r.relation_ptr(0)
        if n:
            self.ctx.bind_device(0, ptr, n, keepalive=self.ctx_r)

    def partition(self, side, params):
        """Partition this rank's R (side 0, on the R stream) or S (side 1) shard."""
        if side == 0:
            return self.ctx_r.partition(0, params)
        return self.ctx.partition(side, params)

    def build_ready(self):
        """Order the main stream after everything enqueued on the R stream."""
        ev = self.torch.cuda.Event()
        ev.record(self.stream_r)
        self.stream.wait_event(ev)

    def pack(self, view, maxn, P):
        """Device copy of a partitioned R view into the packed send layout, on
        the R stream; returns the send tensor once the main stream is ordered
        after it (the all-gather is issued from the main stream)."""
        import ctypes as C
        maxn, E = pack_layout(maxn, P)
        with self.torch.cuda.stream(self.stream_r):
            send = self.tensor(E, self.torch.int64)
        base = send.data_ptr()
        L = self.ctx_r._L
        self.ctx_r._check(L.phj_partitioned_download(self.ctx_r._h, C.byref(view), C.c_void_p(base),
                                                     C.c_void_p(0), C.c_void_p(base + maxn * 8)))
        return send

    def _count(self):
        c = self.torch.zeros(1, dtype=self.torch.int64, device=self.device)
        return c

    def join_packed(self, params, recv, sizes, maxn, P):
        """Build over every rank's gathered shard, probe the local S shard; returns
        the local count as a device tensor (nothing waits on the host)."""
        from ._capi import Partitioned
        maxn, E = pack_layout(maxn, P)
        base = recv.data_ptr()
        segs = []
        for g, n in enumerate(sizes):
            v = Partitioned()
            v.keys = base + (g * E) * 8
            v.payloads = None          # key-only build segments
            v.bounds = base + (g * E + maxn) * 8
            v.n = n
            v.num_partitions = P
            segs.append(v)
        cnt = self._count()
        self.ctx.join_partitioned_async(params, segs, cnt.data_ptr())
        return cnt

    def join_local(self, params, view):
        cnt = self._count()
        self.ctx.join_partitioned_async(params, [view], cnt.data_ptr())
        return cnt

    def timers(self):
        t = {}
        for ctx in (self.ctx_r, self.ctx):
            for name, ms, nbytes in ctx.timers_report().timers():
                a = t.setdefault(name, [0.0, 0])
                a[0] += ms
                a[1] += nbytes
        return [(k, v[0], v[1]) for k, v in t.items()]

    def count_in_range(self, side, lo, hi):
        return (self.ctx_r if side == 0 else self.ctx).count_in_range(side, lo, hi)

    def build_shard(self):
        """This rank's build shard as an (n, 2) int64 device tensor (a view of
        the R context's relation, no copy)."""
        ptr, n = self.ctx_r.relation_ptr(0)

        class _Cai:
            __cuda_array_interface__ = {"shape": (int(n), 2), "typestr": "<i8", "data": (int(ptr or 0), False),
                                        "version": 2, "strides": None}
        if n == 0:
            return self.torch.zeros((0, 2), dtype=self.torch.int64, device=self.device)
        return self.torch.as_tensor(_Cai(), device=self.device)

    def join_nopart_replicated(self, params, full_r):
        """NoPartitioning join of the local S shard against the whole build
        relation `full_r` ((|R|, 2) device tensor); returns the local count
        as a device tensor."""
        self.torch.cuda.current_stream().synchronize()
        self.ctx.bind_device(0, full_r.data_ptr(), full_r.shape[0], keepalive=full_r)
        r = self.ctx.join(params)
        m = r.matches
        self.last_timers = r.timers()
        self.share_build()
        return self.torch.tensor([m], dtype=self.torch.int64, device=self.device)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


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


def distributed_join(engine, params, nR: int, nS: int, rank: int, world: int, dist=None,
                     timers: bool = True, force_exchange: bool = False):
    """Join the range-sharded relations already resident on every rank.

    One step: partition R (R stream); pack it; start the all-gather (RCCL,
    asynchronous); partition S meanwhile (main stream); wait for the gather;
    build + probe; all-reduce the count. The host waits once, for the
    final count. With world == 1 no collective runs unless force_exchange
    (which drives the N>1 branch, RCCL included, on a world of one: the
    one-GPU test of the exchange path). timers=False leaves the
    per-kernel timers accumulating in the engine (read them once, after many
    steps, with engine.timers()).
    """
    torch = engine.torch
    if world == 1 and not force_exchange:
        # no exchange waits on R: issue the long S partition first so the GPU
        # is busy while the host issues R's (small) kernels on the R stream
        if os.environ.get("PHJ_W1_ORDER", "sr") == "rs":
            view = engine.partition(0, params)
            engine.partition(1, params)
        else:
            engine.partition(1, params)
            view = engine.partition(0, params)
        engine.build_ready()
        cnt = engine.join_local(params, view)
        total = local = int(cnt.item())
        return DistResult(matches=total, local_matches=local, timers=engine.timers() if timers else [])
    s_done = engine.partition_async(1, params) if hasattr(engine, "partition_async") else None
    view = engine.partition(0, params)      # R stream
    P = view.num_partitions
    sizes = [hi - lo for lo, hi in (shard_range(nR, r, world) for r in range(world))]
    maxn = max_shard(nR, world)
    send = engine.pack(view, maxn, P)
    # the all-gather waits on R only: issued from the R stream (RCCL runs it on
    # its own stream) before the host spends time issuing the S partition
    side = getattr(engine, "stream_r", None)
    with torch.cuda.stream(side) if side is not None else _null():
        recv = engine.tensor(world * send.numel(), torch.int64)
        work = _all_gather(dist, recv, send)
    if side is not None:
        recv.record_stream(engine.stream)
    if s_done is not None:
        s_done.result()                     # S was issued by the issuer thread meanwhile
    else:
        engine.partition(1, params)         # main stream, beside the exchange
    engine.build_ready()
    if work is not None:
        work.wait()
    cnt = engine.join_packed(params, recv, sizes, maxn, P)
    local = cnt.clone()
    _all_reduce(dist, cnt)
    total = int(cnt.item())
    local = int(local.item())
    return DistResult(matches=total, local_matches=local, timers=engine.timers() if timers else [])


def distributed_join_nopart(engine, params, nR: int, nS: int, rank: int, world: int, dist=None,
                            force_exchange: bool = False):
    """NoPartitioning over range-sharded relations: the build
    relation is replicated with one all-gather of the R shards (padded to the
    largest shard, then compacted), every rank builds the global table
    locally and probes its own S shard, and the counts are summed with an
    all-reduce. S never leaves its GPU. force_exchange runs the collectives
    on a world of one (the one-GPU test of this path)."""
    torch = engine.torch
    shard = engine.build_shard()
    if world == 1 and not force_exchange:
        cnt = engine.join_nopart_replicated(params, shard)
        total = local = int(cnt.item())
        return DistResult(matches=total, local_matches=local, timers=getattr(engine, "last_timers", []))
    sizes = [hi - lo for lo, hi in (shard_range(nR, r, world) for r in range(world))]
    maxn = max(sizes)
    send = shard.new_zeros((maxn, 2))
    send[:shard.shape[0]].copy_(shard)
    recv = shard.new_empty((world * maxn, 2))
    work = _all_gather(dist, recv, send)
    if work is not None:
        work.wait()
    full = torch.cat([recv[g * maxn:g * maxn + sizes[g]] for g in range(world)])
    cnt = engine.join_nopart_replicated(params, full)
    local = cnt.clone()
    _all_reduce(dist, cnt)
    return DistResult(matches=int(cnt.item()), local_matches=int(local.item()),
                      timers=getattr(engine, "last_timers", []))


def unpack_segments_numpy(recv, sizes, maxn, P):
    """Split a gathered packed buffer back into per-rank (keys, bounds)."""
    maxn, E = pack_layout(maxn, P)
    recv = np.asarray(recv)
    segs = []
    for g, n in enumerate(sizes):
        blk = recv[g * E:(g + 1) * E]
        bounds = blk[maxn:].view(np.uint32)[:P + 1].astype(np.int64)
        segs.append((blk[:n], bounds))
    return segs
