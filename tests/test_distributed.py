"""The multi-GPU member step's host protocol over gloo on CPU (world 2-3).

The join itself is C++/HIP in libphj_hip.so (csrc/phj_group.h) and needs a
GPU; what crosses the ranks is defined by the library's host-only functions,
which phj_group.h itself calls and these tests drive through the C ABI:
  * phj_shard_range: rows of each rank (range shards, §8(e));
  * phj_exchange_layout: one rank's all-gathered block, build codes in final
    partition order | zero padding | bounds[P + 1] (uint32);
  * phj_count_contribution / phj_count_verdict: the {count, failed} words of
    the count all-reduce and the global count (or PHJ_ERR_STATE) they give.
Each rank's packed block is built by tests/exchange_proto.py from the oracle's
hash codes by the library's rules (phj_exchange_geometry: the segments --
the LDS join's clusters or the final partitions; phj_exchange_layout: the
block), and its table probe is the oracle's (test infrastructure). So only
the geometry, the layout arithmetic and the count reduction are the library's
here; the library's own pack (the device step) is compared with the same
restatement by tests/test_gpu_multirank.py::test_member_pack_matches_protocol.
This checks that blocks packed and read by those rules carry every rank's
build side intact, that the reduction counts what
the reference counts (the semi-join, src/RadixCluster/HashJoin.hpp:295-301),
and that one failed rank (an all-zero block, failed word 1) makes every rank
report the failure while its block still reads as a valid empty segment.
The reference's parallel split is a thread pool (src/main.cpp:235-241).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import partitionedhashjoin_amd as phj
import exchange_proto as X
from oracle import oracle as O


def _tables(nR, nS, alpha, seed):
    R, S = O.generate_tables(nR, nS, alpha, seed, threads=2)
    S[::5, 0] += nR  # a fifth of the probe keys miss
    return R, S


def _worker(rank, world, port, nR, nS, alpha, seed, bits, nparts, fail_rank, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        R, S = _tables(nR, nS, alpha, seed)
        params = phj.radix_params(bits, num_partitions=nparts, hash=phj.HASH_MURMUR3, seed=1234)
        P, segment_of = X.geometry(params, nR)   # the library's segments: clusters or final partitions
        rlo, rhi = phj.shard_range(nR, rank, world)
        slo, shi = phj.shard_range(nS, rank, world)
        # every rank's real shard size first (phj_group.h exchange_sizes)
        sizes = torch.zeros(world, dtype=torch.int64)
        dist.all_gather_into_tensor(sizes, torch.tensor([rhi - rlo], dtype=torch.int64))
        codes_elems, block_elems = phj.exchange_layout(int(sizes.max()), P)
        failed = rank == fail_rank
        send = np.zeros(block_elems, dtype=np.int64) if failed else X.pack(R[rlo:rhi], params, nR, codes_elems, block_elems)
        recv = torch.zeros(world * block_elems, dtype=torch.int64)
        dist.all_gather_into_tensor(recv, torch.from_numpy(send))
        segs = X.segments(recv.numpy(), world, P, codes_elems, block_elems)
        for g, (codes, b) in enumerate(segs):
            # segment-major with consistent bounds; a failed rank's block is empty
            assert b[0] == 0 and np.all(np.diff(b) >= 0)
            assert codes.shape[0] == (0 if g == fail_rank else int(sizes[g]))
            assert np.array_equal(segment_of(codes), np.repeat(np.arange(P), np.diff(b)))
        kind = O.HASH_MURMUR3
        build = np.concatenate([c for c, _ in segs])
        local = O.semijoin_count_keys(build, O.hash_keys(kind, S[slo:shi, 0], 1234).view(np.int64))
        words = torch.from_numpy(phj.count_contribution(local, failed).view(np.int64).copy())
        dist.all_reduce(words)
        try:
            out[rank] = ("ok", phj.count_verdict(words.numpy().view(np.uint64)), local)
        except phj.PhjError as e:
            out[rank] = ("error", e.code, local)
    finally:
        dist.destroy_process_group()


def _np_worker(rank, world, port, nR, nS, out):
    # NoPartitioning (§8(e)): every rank's R shard broadcast to all (an
    # all-gather-v into one contiguous relation, phj_group.h member_nopart), the
    # global table built and the local S shard probed, the counts reduced
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        R, S = _tables(nR, nS, 1.25, 9)
        parts = []
        for g in range(world):
            lo, hi = phj.shard_range(nR, g, world)
            t = torch.from_numpy(np.ascontiguousarray(R[lo:hi])) if g == rank else torch.zeros((hi - lo, 2), dtype=torch.int64)
            dist.broadcast(t, src=g)
            parts.append(t.numpy())
        full = np.concatenate(parts)
        slo, shi = phj.shard_range(nS, rank, world)
        local = O.join_nopart(full, S[slo:shi]).matches
        words = torch.from_numpy(phj.count_contribution(local).view(np.int64).copy())
        dist.all_reduce(words)
        out[rank] = ("ok", phj.count_verdict(words.numpy().view(np.uint64)), local)
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


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 10_000_000):
        for w in (1, 2, 3, 8):
            rs = [phj.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1


def test_exchange_layout():
    # codes padded to 64 elements (16-B aligned columns), then P + 1 uint32 bounds
    for maxn in (0, 1, 63, 64, 65, 1_250_000):
        for P in (1, 2, 32, 65536, 4_194_304):
            ce, be = phj.exchange_layout(maxn, P)
            assert ce % 64 == 0 and maxn <= ce < maxn + 64
            assert 2 * (be - ce) >= P + 1 and 2 * (be - ce) <= P + 2


def test_count_words():
    assert list(phj.count_contribution(123)) == [123, 0]
    assert list(phj.count_contribution(123, failed=True)) == [0, 1]
    assert phj.count_verdict([5, 0]) == 5
    with pytest.raises(phj.PhjError) as e:
        phj.count_verdict([5, 2])
    assert e.value.code == phj._capi.PHJ_ERR_STATE


@pytest.mark.parametrize("world,bits,nparts", [(2, (4, 4), 0), (3, (6, 0), 0), (2, (1, 0), 37)])
def test_member_protocol_gloo(world, bits, nparts):
    nR, nS, alpha, seed = 20_011, 150_007, 1.25, 3
    R, S = _tables(nR, nS, alpha, seed)
    expect = O.semijoin_count(R, S)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), nR, nS, alpha, seed, bits, nparts, -1, out), nprocs=world)
    assert {out[r][:2] for r in range(world)} == {("ok", expect)}
    assert sum(out[r][2] for r in range(world)) == expect


def test_member_protocol_failure_gloo():
    # rank 1 fails before the all-gather: it sends an all-zero block (peers
    # read an empty build segment) and the failed word; every rank then
    # reports PHJ_ERR_STATE instead of a count
    world, nR, nS = 3, 20_011, 150_007
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), nR, nS, 1.05, 4, (4, 4), 0, 1, out), nprocs=world)
    assert {out[r][:2] for r in range(world)} == {("error", phj._capi.PHJ_ERR_STATE)}


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_nopart_gloo(world):
    nR, nS = 20_001, 150_007
    R, S = _tables(nR, nS, 1.25, 9)
    expect = O.semijoin_count(R, S)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_np_worker, args=(world, _free_port(), nR, nS, out), nprocs=world)
    assert {out[r][:2] for r in range(world)} == {("ok", expect)}
    assert sum(out[r][2] for r in range(world)) == expect
