"""Multi-GPU join: thin callers of the C ABI's multi-device contexts, and the
CPU rehearsal of the same step.

The reference is single-process (no distributed runtime); this
layer follows BASELINE.json's north star. The join itself lives in
libphj_hip.so (csrc/phj_group.h): both relations are range-sharded across the
ranks, every rank radix-partitions its R and S shards, the partitioned build
keys are exchanged with one RCCL all-gather over xGMI (the only data-path
collective: S, 95% of the bytes, never leaves its GPU and stays balanced under
any key skew), each rank joins its S shard against the gathered build side and
the counts are summed with an RCCL all-reduce. NoPartitioning replicates R
(an all-gather-v) and probes the local S shard.

Two ways to run it, both one C call per join:
  * one process driving several GPUs: `Context(devices=[0, 1, ...])`;
  * one process per GPU (torchrun, bench.py --gpus N): `rank_context`, which
    only hands rank 0's RCCL unique id to the other ranks over
    torch.distributed and creates the rank's context (phj_ctx_create_rank).

`distributed_join` / `distributed_join_nopart` restate the per-rank step over
torch.distributed collectives for an engine interface; the CPU tests run them
with an oracle engine over gloo (world 2-3), so the sharding, the exchange
layout (padded key blocks | bounds, the real shard sizes gathered first) and
the count reduction are covered without a GPU.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import Context, comm_unique_id, CTX_EXCHANGE


def shard_range(n: int, rank: int, world: int):
    """Rows [lo, hi) of an n-row relation held by `rank`: the range sharding
    every multi-device context applies (phj_shard_range, csrc/phj_group.h
    shard_range; tests/test_distributed.py pins the two together). Pure Python,
    so the CPU rehearsal needs no HIP runtime."""
    if not 0 <= rank < world:
        return (0, 0)
    return ((n * rank) // world, (n * (rank + 1)) // world)


def max_shard(n: int, world: int) -> int:
    return max(hi - lo for lo, hi in (shard_range(n, r, world) for r in range(world)))


def pack_layout(maxn: int, P: int):
    """int64 elements of one rank's exchange block: keys[maxn] | bounds[P+1]
    (uint32, two per element), maxn padded to 64 elements (csrc/phj_group.h
    PackLayout). Only the keys travel: the join tests key equality and never
    reads a build payload (RadixCluster/HashJoin.hpp:295-301)."""
    maxn = (maxn + 63) // 64 * 64
    return maxn, maxn + (P + 2) // 2


@dataclass
class DistResult:
    matches: int             # global semi-join count (all-reduced)
    local_matches: int
    timers: list             # this rank's per-kernel device timers (name, ms, bytes)


# ---- the GPU path: multi-device contexts ----

def rank_context(local_rank: int, rank: int, world: int, dist=None, exchange: bool = False) -> Context:
    """This rank's context. world > 1: one device of a multi-process job
    (phj_ctx_create_rank; rank 0's RCCL unique id is broadcast over `dist`).
    world == 1: a single-device context, or with `exchange` the multi-GPU path
    on a world of one (RCCL collectives included)."""
    if world == 1:
        if exchange:
            return Context(devices=[local_rank], flags=CTX_EXCHANGE)
        return Context(local_rank)
    box = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return Context.rank(local_rank, world, rank, box[0])


def generate_shards(ctx: Context, nR: int, nS: int, alpha: float, seed: int, rank: int, world: int,
                    start: int = 1):
    """The rank's rows of generateTables (src/main.cpp:35-79): R Sequential
    from `start`, S Zipf over [1, |R|]; on a multi-process context every rank
    calls this (the relation calls are collective)."""
    _, _, nlocal = ctx.info()
    w = world if nlocal == 1 else 1      # a context with all devices takes whole relations
    r = rank if nlocal == 1 else 0
    rlo, rhi = shard_range(nR, r, w)
    slo, shi = shard_range(nS, r, w)
    ctx.generate_sequential(0, rhi - rlo, start, rlo)
    ctx.generate_zipf(1, shi - slo, alpha, 1, nR, seed, slo)


# ---- the step over torch.distributed (CPU rehearsal with an engine) ----

def _all_gather(dist, out, inp):
    dist.all_gather_into_tensor(out, inp)


def _all_reduce(dist, t):
    dist.all_reduce(t)


def distributed_join(engine, params, nR: int, nS: int, rank: int, world: int, dist=None):
    """The member step of csrc/phj_group.h over torch.distributed: partition
    the R shard, all-gather the real shard sizes, pack keys | bounds into
    padded blocks, all-gather them, join the local S shard against every
    block, all-reduce the count."""
    torch = engine.torch
    view = engine.partition(0, params)
    engine.partition(1, params)
    if world == 1:
        cnt = engine.join_local(params, view)
        m = int(cnt.item())
        return DistResult(matches=m, local_matches=m, timers=engine.timers())
    P = view.num_partitions
    # the real shard sizes (not the nominal ranges: a caller may bind its own shards)
    n_local = torch.tensor([view.n], dtype=torch.int64)
    sizes_t = torch.zeros(world, dtype=torch.int64)
    _all_gather(dist, sizes_t, n_local)
    sizes = [int(x) for x in sizes_t]
    maxn = max(sizes)
    send = engine.pack(view, maxn, P)
    recv = engine.tensor(world * send.numel(), torch.int64)
    _all_gather(dist, recv, send)
    cnt = engine.join_packed(params, recv, sizes, maxn, P)
    local = int(cnt.item())
    _all_reduce(dist, cnt)
    return DistResult(matches=int(cnt.item()), local_matches=local, timers=engine.timers())


def distributed_join_nopart(engine, params, nR: int, nS: int, rank: int, world: int, dist=None):
    """NoPartitioning over range shards (§8(e)): the R shards are gathered
    (all-gather-v: real sizes first, padded blocks, compacted), every rank
    builds the global table and probes its S shard, the counts are summed."""
    torch = engine.torch
    shard = engine.build_shard()
    if world == 1:
        cnt = engine.join_nopart_replicated(params, shard)
        m = int(cnt.item())
        return DistResult(matches=m, local_matches=m, timers=[])
    sizes_t = torch.zeros(world, dtype=torch.int64)
    _all_gather(dist, sizes_t, torch.tensor([shard.shape[0]], dtype=torch.int64))
    sizes = [int(x) for x in sizes_t]
    maxn = max(sizes)
    send = shard.new_zeros((maxn, 2))
    send[:shard.shape[0]].copy_(shard)
    recv = shard.new_empty((world * maxn, 2))
    _all_gather(dist, recv, send)
    full = torch.cat([recv[g * maxn:g * maxn + sizes[g]] for g in range(world)])
    cnt = engine.join_nopart_replicated(params, full)
    local = int(cnt.item())
    _all_reduce(dist, cnt)
    return DistResult(matches=int(cnt.item()), local_matches=local, timers=[])


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
