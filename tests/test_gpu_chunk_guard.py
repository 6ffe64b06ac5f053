"""A stale chunk table must yield an error code, never a write through it.

Round 4's GPU fault (VERDICT r04 "What's weak" 1): a regrown chunk table at
the same address kept another buffer's bytes, and the chunked pass 1 read
them as published chunk ids and stored tuples through them. The chunked
passes (k_chunk_codes, k_scatter_chunked) and k_tile_chunks now bound-check
every chunk id and chain index they read back (phj_partition.h chunk_err_word);
here the table is poisoned deterministically through the test hook
phj_debug_poison_chunk_table before a join, which must return PHJ_ERR_STATE
(no fault), and the next join must be exact again (the table is cleared).
Reference: the scatter this replaces, src/RadixCluster/HashJoin.hpp:394-412.
"""
import numpy as np
import pytest

import partitionedhashjoin_amd as phj
from partitionedhashjoin_amd import PhjError

pytestmark = pytest.mark.gpu

PHJ_ERR_STATE = -4


def _relations(ctx, nR, nS, alpha=1.05, seed=77):
    ctx.generate_sequential(phj.SIDE_BUILD, nR, 1)
    ctx.generate_zipf(phj.SIDE_PROBE, nS, alpha, 1, nR, seed)
    S = ctx.download(phj.SIDE_PROBE)
    S[::5, 0] = -S[::5, 0]   # misses
    ctx.upload(phj.SIDE_PROBE, S)
    return int(np.count_nonzero(S[:, 0] > 0))


@pytest.mark.parametrize("byte", [0xFF, 0x01])
def test_poisoned_chunk_table_returns_error_then_recovers(ctx, byte):
    """On-chip join (S's keys-only chunked pass 1): 0xFF entries read as
    published chunks with ids far outside the pool, 0x01 entries as published
    chunk 0x01010101 (outside every shard's pool)."""
    expect = _relations(ctx, 200_000, 3_000_000)
    params = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3)
    assert ctx.join(params).matches == expect
    ctx.debug_poison_chunk_table(phj.SIDE_PROBE, params, byte)
    with pytest.raises(PhjError) as e:
        ctx.join(params)
    assert e.value.code == PHJ_ERR_STATE
    assert "stale" in str(e.value)
    # the table was cleared: exact again, twice
    assert ctx.join(params).matches == expect
    assert ctx.join(params).matches == expect


def test_poisoned_chunk_table_payload_pass(chunk_ctx):
    """The whole-tuple chunked pass 1 (k_scatter_chunked, unordered
    partitions of phj_partition): the poisoned pass reports PHJ_ERR_STATE when
    its output is read back, and the next partition is exact."""
    c = chunk_ctx
    nR, nS = 100_000, 2_000_000
    _relations(c, nR, nS)
    params = phj.radix_params((6, 6), hash=phj.HASH_XXH3)
    ref = c.partition(phj.SIDE_PROBE, params)
    k0, p0, b0 = c.download_partitioned(ref)
    c.debug_poison_chunk_table(phj.SIDE_PROBE, params, 0xFF)
    v = c.partition(phj.SIDE_PROBE, params)
    with pytest.raises(PhjError) as e:
        c.download_partitioned(v)
    assert e.value.code == PHJ_ERR_STATE
    v = c.partition(phj.SIDE_PROBE, params)
    k1, p1, b1 = c.download_partitioned(v)
    assert np.array_equal(b0, b1)
    for p in range(len(b0) - 1):   # unordered inside a partition: compare as multisets
        lo, hi = b0[p], b0[p + 1]
        assert np.array_equal(np.sort(k0[lo:hi]), np.sort(k1[lo:hi]))


# ---- round 6: r05a's stale-table report, pinned ----
#
# VERDICT r05 "What's weak" 1: gpurun_out/r05a.out:32 (an early round-5 build)
# failed test_full_size_eight_members[nopart-xxh3-s1.05-x8] on a fresh
# 8-member context after the C3 / C5 cases with "device 1: chunked pass 1 read
# a chunk-table entry out of range (stale table, error bits 0)". Error bits 0
# means no pass raised its error word: the report came from the host reading
# word 1 of the member's count pair as "the probe folded a pass-1 error". The
# NoPartitioning member step copies only its 8-byte count into that pair
# (allreduce_count, pair = false), so word 1 was whatever the freshly allocated
# buffer held -- here, the previous test's freed context's bytes. That build's
# read_count tested word 1 on every local join; it now reads it only for the
# radix step's {count, failed} pair (phj_group.h read_count, `pair`). The hook
# phj_debug_poison_alloc makes "whatever the buffer held" deterministic: every
# new workspace buffer starts as `byte`, so any word read before it is written
# shows, on every join path, in the r05a order and on fresh members.

NR_G, NS_G, SHIFT_G = 1_000_000, 16_000_000, 3


def _group_relations(g, alpha=1.05, seed=4242):
    g.generate_sequential(phj.SIDE_BUILD, NR_G, 1 + SHIFT_G)
    g.generate_zipf(phj.SIDE_PROBE, NS_G, alpha, 1, NR_G, seed)
    S = g.download(phj.SIDE_PROBE, NS_G)
    S[::7, 0] = -S[::7, 0]
    g.upload(phj.SIDE_PROBE, S)
    keys = S[:, 0]
    return int(np.count_nonzero((keys > SHIFT_G) & (keys <= NR_G + SHIFT_G)))


R05A_ORDER = [   # (name, params, Zipf skew): test_gpu_fullsize_group.py's cases in order
    ("C3-radix-8+8-murmur3", lambda: phj.radix_params((8, 8), hash=phj.HASH_MURMUR3), 1.05),
    ("C5-radix-8+8-murmur3", lambda: phj.radix_params((8, 8), hash=phj.HASH_MURMUR3), 1.25),
    ("nopart-xxh3", lambda: phj.nopart_params(hash=phj.HASH_XXH3), 1.05),
]


@pytest.mark.parametrize("byte", [0xFF, 0x01])
def test_r05a_sequence_fresh_members_poisoned(byte):
    """The r05a order (radix x8, radix x8, then NoPartitioning x8), each on a
    fresh 8-member local context whose every allocation starts as `byte`:
    every join exact. Fails on the r05a build's read_count (word 1 tested on
    the NoPartitioning step, whose pair it never writes)."""
    for name, mk, alpha in R05A_ORDER:
        with phj.Context(devices=[0] * 8, flags=phj.CTX_LOCAL) as g:
            g.debug_poison_alloc(byte)
            expect = _group_relations(g, alpha)
            assert 0.3 * NS_G < expect < 0.9 * NS_G
            for _ in range(2):
                assert g.join(mk()).matches == expect, name


def test_poisoned_alloc_every_kind_on_one_group():
    """One poisoned 8-member context running every kind back to back (the
    NoPartitioning step first, then radix, then NoPartitioning again)."""
    with phj.Context(devices=[0] * 8, flags=phj.CTX_LOCAL) as g:
        g.debug_poison_alloc(0xFF)
        expect = _group_relations(g)
        for name, mk, _ in [R05A_ORDER[2]] + R05A_ORDER + [R05A_ORDER[0]]:
            assert g.join(mk()).matches == expect, name


def test_poisoned_alloc_rccl_world_of_one():
    """The RCCL member step (world of one) with poisoned buffers."""
    with phj.Context(devices=[0], flags=phj.CTX_EXCHANGE) as g:
        g.debug_poison_alloc(0xFF)
        expect = _group_relations(g)
        for name, mk, _ in [R05A_ORDER[2], R05A_ORDER[0], R05A_ORDER[2]]:
            assert g.join(mk()).matches == expect, name


def test_poisoned_alloc_one_device_every_path():
    """A fresh single-device context with every allocation poisoned: the LDS
    join (plain and under the bench's DEFER|LEAN timers), the reference's
    `-p 1024` hash % P plan, the bucket-chained table kind, NoPartitioning,
    and the materialised join's row count."""
    with phj.Context(0) as c:
        c.debug_poison_alloc(0xFF)
        expect = _relations(c, 500_000, 8_000_000)
        radix = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3)
        timed = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3)
        timed.flags = radix.flags | phj.DEFER_TIMERS | phj.LEAN_TIMERS
        for p in (radix, timed, timed, phj.radix_params(num_partitions=1024, hash=phj.HASH_XXH3),
                  phj.radix_params((8, 8), hash=phj.HASH_XXH3, chained=True),
                  phj.nopart_params(hash=phj.HASH_XXH3), radix):
            assert c.join(p).matches == expect
        c.timers_report()
        assert c.join_materialize(radix).matches == expect
