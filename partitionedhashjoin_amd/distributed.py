"""Multi-GPU join: thin callers of the C ABI's multi-device contexts.

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

The exchange layout and the count reduction the member step applies are the
library's own host-only functions (phj_exchange_layout, phj_count_contribution,
phj_count_verdict, include/phj.h); tests/test_distributed.py drives them over
gloo on CPU (world 2-3).
"""
from __future__ import annotations

from . import Context, comm_unique_id, CTX_EXCHANGE, shard_range


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
