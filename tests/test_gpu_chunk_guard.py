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
