"""Multi-rank orchestration (partitionedhashjoin_amd/distributed.py) over gloo
on CPU: range sharding, partitioned build-shard all-gather, per-rank join,
count all-reduce. A test-only engine computes each rank's partitions with the
oracle, so this exercises exactly the collective layout the HIP engine uses
(fixed-size padded shards, per-shard partition bounds) without a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import partitionedhashjoin_amd as phj
from oracle import oracle as O
from partitionedhashjoin_amd.distributed import (distributed_join, distributed_join_nopart, max_shard, pack_layout, shard_range,
                                                 unpack_segments_numpy)


class _View:
    def __init__(self, keys, pays, bounds, P):
        self.keys, self.pays, self.bounds = keys, pays, bounds
        self.n = keys.shape[0]
        self.num_partitions = P


class OracleShardEngine:
    """CPU stand-in for HipShardEngine with the same interface (test infrastructure)."""

    def __init__(self, R, S):
        self.torch = torch
        self.rel = {0: R, 1: S}
        self.views = {}

    @staticmethod
    def _geometry(p):
        if p.num_partitions:
            return int(p.num_partitions), False
        return 1 << (p.radix_bits[0] + p.radix_bits[1]), True

    def tensor(self, n, dtype):
        return torch.zeros(int(n), dtype=dtype)

    def partition(self, side, params):
        P, radix = self._geometry(params)
        out, bounds = O.partition(self.rel[side], P, radix, params.hash, params.hash_seed, workers=2)
        v = _View(out[:, 0].copy(), out[:, 1].copy(), bounds, P)
        self.views[side] = v
        return v

    def pack(self, v, maxn, P):
        maxn, E = pack_layout(maxn, P)
        buf = np.zeros(E, dtype=np.int64)
        buf[:v.n] = v.keys
        buf[maxn:].view(np.uint32)[:P + 1] = v.bounds.astype(np.uint32)
        return torch.from_numpy(buf)

    def _count(self, params, segs):
        P, radix = self._geometry(params)
        for keys, bounds in segs:
            # every gathered shard arrives partition-major with consistent bounds
            q = O.partition_ids(keys, P, radix, params.hash, params.hash_seed).astype(np.int64)
            expect = np.repeat(np.arange(P), np.diff(bounds.astype(np.int64)))
            assert np.array_equal(q, expect)
        rkeys = np.concatenate([k for k, _ in segs]) if segs else np.zeros(0, dtype=np.int64)
        return torch.tensor([O.semijoin_count_keys(rkeys, self.views[1].keys)], dtype=torch.int64)

    def join_packed(self, params, recv, sizes, maxn, P):
        return self._count(params, unpack_segments_numpy(recv.numpy(), sizes, maxn, P))

    def join_local(self, params, v):
        return self._count(params, [(v.keys, v.bounds)])

    def timers(self):
        return []

    def build_shard(self):
        return torch.from_numpy(np.ascontiguousarray(self.rel[0]))

    def join_nopart_replicated(self, params, full_r):
        R = full_r.numpy()
        return torch.tensor([O.join_nopart(R, self.rel[1]).matches], dtype=torch.int64)

    def build_ready(self):
        pass


def _tables(nR, nS, alpha, seed):
    R, S = O.generate_tables(nR, nS, alpha, seed, threads=2)
    S[::5, 0] += nR  # a fifth of the probe keys miss
    return R, S


def _worker(rank, world, port, nR, nS, alpha, seed, bits, nparts, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        R, S = _tables(nR, nS, alpha, seed)
        rlo, rhi = shard_range(nR, rank, world)
        slo, shi = shard_range(nS, rank, world)
        eng = OracleShardEngine(R[rlo:rhi], S[slo:shi])
        p = phj.radix_params(bits, num_partitions=nparts, hash=phj.HASH_MURMUR3, seed=1234)
        res = distributed_join(eng, p, nR, nS, rank, world, dist)
        out[rank] = (res.matches, res.local_matches)
    finally:
        dist.destroy_process_group()


def _np_worker(rank, world, port, nR, nS, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        R, S = _tables(nR, nS, 1.25, 9)
        rlo, rhi = shard_range(nR, rank, world)
        slo, shi = shard_range(nS, rank, world)
        eng = OracleShardEngine(R[rlo:rhi], S[slo:shi])
        res = distributed_join_nopart(eng, phj.nopart_params(), nR, nS, rank, world, dist)
        out[rank] = (res.matches, res.local_matches)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_library_shard_range_is_the_documented_split():
    # phj_shard_range (host-only C ABI) = rows [n*r/G, (n*(r+1))/G), exact for any n
    for n in (0, 1, 7, 10_000_000, 2**40 + 3, 2**63):
        for w in (1, 2, 3, 7, 8, 16):
            for r in range(w):
                assert phj.shard_range(n, r, w) == ((n * r) // w, (n * (r + 1)) // w)
    assert phj.shard_range(10, 3, 2) == (0, 0)   # out of range rank: empty
    # the pure-Python helper of the CPU rehearsal is the same split
    for n in (0, 1, 7, 10_000_000, 2**40 + 3):
        for w in (1, 3, 8):
            for r in range(w + 1):
                assert shard_range(n, r, w) == phj.shard_range(n, r, w)


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 10_000_000):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max_shard(n, w) - min(hi - lo for lo, hi in rs) <= 1


@pytest.mark.parametrize("world,bits,nparts", [(2, (4, 4), 0), (3, (6, 0), 0), (2, (1, 0), 37)])
def test_distributed_join_gloo(world, bits, nparts):
    nR, nS, alpha, seed = 20_011, 150_007, 1.25, 3
    R, S = _tables(nR, nS, alpha, seed)
    expect = O.semijoin_count(R, S)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), nR, nS, alpha, seed, bits, nparts, out), nprocs=world)
    totals = {out[r][0] for r in range(world)}
    assert totals == {expect}
    assert sum(out[r][1] for r in range(world)) == expect


def test_single_rank_path():
    R, S = _tables(5000, 40_000, 1.05, 8)
    eng = OracleShardEngine(R, S)
    res = distributed_join(eng, phj.radix_params((3, 3)), 5000, 40_000, 0, 1, None)
    assert res.matches == O.semijoin_count(R, S)


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_nopart_gloo(world):
    nR, nS = 20_001, 150_007
    R, S = _tables(nR, nS, 1.25, 9)
    expect = O.semijoin_count(R, S)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_np_worker, args=(world, _free_port(), nR, nS, out), nprocs=world)
    assert {out[r][0] for r in range(world)} == {expect}
    assert sum(out[r][1] for r in range(world)) == expect
