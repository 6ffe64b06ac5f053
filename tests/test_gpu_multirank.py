"""The multi-GPU join behind the C ABI (csrc/phj_group.h) on one GPU.

* PHJ_CTX_LOCAL: 2-3 members on device 0 driven by their own threads, the
  exchange done by device copies (RCCL refuses two ranks per device): the
  whole multi-member step (range shards, R partition + pack, gather,
  multi-segment join, count sum; replicated NoPartitioning build) runs.
* PHJ_CTX_EXCHANGE: the same step with the RCCL collectives on a world of one
  (ncclCommInitAll), and phj_ctx_create_rank with a unique id (ncclCommInitRank,
  the size all-gather of the multi-process path).
The 8-GPU bench runs exactly this code with more ranks.

Workloads have a real miss fraction: R holds keys [1 + off, |R| + off], S is
Zipf over [1, |R|], so the S keys below 1 + off miss (the hottest keys).
"""
import numpy as np
import pytest

import partitionedhashjoin_amd as phj
from partitionedhashjoin_amd import shard_range
from partitionedhashjoin_amd.distributed import generate_shards
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED = 0x1234_5678_9ABC_DEF1
PARAMS = [("radix-8+8-murmur3", phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED)),
          ("radix-mod1024-xxh3", phj.radix_params(num_partitions=1024, hash=phj.HASH_XXH3, seed=SEED)),
          ("nopart-xxh3", phj.nopart_params(hash=phj.HASH_XXH3, seed=SEED))]


def _generate(ctx, nR, nS, alpha, off, rank=0, world=1):
    generate_shards(ctx, nR, nS, alpha, 77, rank, world, start=1 + off)
    return ctx.count_in_range(phj.SIDE_PROBE, 1 + off, nR)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_local_group_on_one_gpu(world):
    nR, nS, off = 300_001, 4_000_003, 100_000
    with phj.Context(devices=[0] * world, flags=phj.CTX_LOCAL) as g:
        assert g.info() == (world, 0, world)
        expect = _generate(g, nR, nS, 1.25, off)
        assert 0 < expect < nS
        for name, p in PARAMS:
            for _ in range(2):   # a second step reuses every buffer
                r = g.join(p)
                assert r.matches == expect, name
            assert r.total_ms > 0 and r.exchange_ms >= 0
            assert "exchange" in {t for t, _, _ in r.timers()}, name


def test_local_group_matches_oracle_on_host_relations():
    # host relations range-sharded on upload; adversarial keys
    rng = np.random.default_rng(5)
    R = np.stack([rng.integers(-50_000, 50_000, 70_001, dtype=np.int64), np.arange(70_001)], axis=1)
    S = np.stack([rng.integers(-100_000, 100_000, 900_007, dtype=np.int64), np.arange(900_007)], axis=1)
    expect = O.semijoin_count(R, S)
    with phj.Context(devices=[0, 0, 0], flags=phj.CTX_LOCAL) as g:
        g.upload(phj.SIDE_BUILD, R)
        g.upload(phj.SIDE_PROBE, S)
        assert np.array_equal(g.download(phj.SIDE_PROBE), S)
        for name, p in PARAMS:
            g.prepare(p)
            assert g.join(p).matches == expect, name


def test_group_shards_concatenate_to_the_single_device_relation():
    n = 4096 * 5 + 123
    with phj.Context(0) as one, phj.Context(devices=[0, 0, 0], flags=phj.CTX_LOCAL) as g:
        one.generate_zipf(1, n, 1.05, 1, 10_000, 9)
        g.generate_zipf(1, n, 1.05, 1, 10_000, 9)
        assert np.array_equal(one.download(1), g.download(1))
        # and a shard generated on its own is the same rows
        lo, hi = shard_range(n, 1, 3)
        one.generate_zipf(1, hi - lo, 1.05, 1, 10_000, 9, lo)
        assert np.array_equal(one.download(1), g.download(1)[lo:hi])


def test_building_blocks_refused_on_several_local_devices():
    with phj.Context(devices=[0, 0], flags=phj.CTX_LOCAL) as g:
        g.upload(phj.SIDE_PROBE, np.zeros((10, 2), dtype=np.int64))
        with pytest.raises(phj.PhjError, match="multi-device"):
            g.partition(phj.SIDE_PROBE, phj.radix_params((4, 0)))
        with pytest.raises(phj.PhjError, match="single-device"):
            g.join_materialize(phj.radix_params((4, 0)))


def test_rccl_world_of_one_group():
    nR, nS, off = 1_000_003, 20_000_001, 250_000
    with phj.Context(devices=[0], flags=phj.CTX_EXCHANGE) as g:
        expect = _generate(g, nR, nS, 1.05, off)
        assert 0 < expect < nS
        for name, p in PARAMS:
            got = [g.join(p).matches for _ in range(3)]
            assert got == [expect] * 3, name


def test_rccl_rank_context_world_of_one():
    # phj_ctx_create_rank: ncclCommInitRank from a unique id, the collective
    # size exchange on every relation call, then the member step
    nR, nS, off = 500_009, 6_000_011, 3
    uid = phj.comm_unique_id()
    assert len(uid) == 128
    with phj.Context.rank(0, 1, 0, uid) as ctx:
        assert ctx.info() == (1, 0, 1)
        expect = _generate(ctx, nR, nS, 1.25, off, rank=0, world=1)
        assert 0 < expect < nS
        for name, p in PARAMS:
            assert ctx.join(p).matches == expect, name
        # PHJ_DEFER_TIMERS on a rank context: the member keeps its timers,
        # timers_report sums them (bench.py's timed loop at N > 1)
        p = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3)
        single = {n for n, _, _ in ctx.join(p).timers()}
        q = type(p).from_buffer_copy(p)
        q.flags = p.flags | phj.DEFER_TIMERS
        ctx.timers_report()
        for _ in range(2):
            r = ctx.join(q)
            assert r.matches == expect and list(r.timers()) == []
        summed = {n: ms for n, ms, _ in ctx.timers_report().timers()}
        assert "exchange" in summed and set(summed) == single and all(ms >= 0 for ms in summed.values())
        # a one-device rank context also takes the building blocks
        v = ctx.partition(phj.SIDE_PROBE, phj.radix_params((8, 8)))
        assert v.n == nS


def test_rehearsal_member_zero_joins_its_shard(monkeypatch):
    # PHJ_REHEARSE (scripts/rehearse_world.py): members > 0 only feed the
    # exchange, so the reported count is member 0's S shard against all of R
    monkeypatch.setenv("PHJ_REHEARSE", "1")
    R, S = O.generate_tables(50_000, 600_001, 1.05, 5, threads=4)
    R[:, 0] += 7
    S[::5, 0] = -S[::5, 0]
    world = 3
    lo, hi = shard_range(S.shape[0], 0, world)
    expect = O.semijoin_count(R, S[lo:hi])
    with phj.Context(devices=[0] * world, flags=phj.CTX_LOCAL) as g:
        g.upload(phj.SIDE_BUILD, R)
        g.upload(phj.SIDE_PROBE, S)
        p = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED)
        for _ in range(3):   # members > 0 pack once, then only take part in the exchange
            assert g.join(p).matches == expect


PHJ_ERR_STATE = -4


@pytest.mark.parametrize("name,p", PARAMS, ids=[a for a, _ in PARAMS])
@pytest.mark.parametrize("world", [2, 3])
def test_local_group_member_failure(world, name, p):
    """A member that fails before the exchange (phj_debug_fail_member): every
    member returns PHJ_ERR_STATE through the local exchange's barrier, no
    fault, and the next join is exact."""
    nR, nS, off = 200_003, 2_000_003, 1_000
    with phj.Context(devices=[0] * world, flags=phj.CTX_LOCAL) as g:
        expect = _generate(g, nR, nS, 1.05, off)
        assert g.join(p).matches == expect
        g.debug_fail_member(world - 1)
        with pytest.raises(phj.PhjError) as e:
            g.join(p)
        assert e.value.code == PHJ_ERR_STATE
        assert g.join(p).matches == expect


@pytest.mark.parametrize("name,p", PARAMS, ids=[a for a, _ in PARAMS])
def test_rccl_world_of_one_failed_rank(name, p):
    """The RCCL failure branch on a world of one: the failed rank still takes
    part in the all-gather with a zeroed block (a valid empty segment) and in
    the count all-reduce with {0, 1}; the join returns PHJ_ERR_STATE, the
    communicator stays usable, the next join is exact."""
    nR, nS, off = 200_003, 2_000_003, 1_000
    with phj.Context(devices=[0], flags=phj.CTX_EXCHANGE) as g:
        expect = _generate(g, nR, nS, 1.05, off)
        assert g.join(p).matches == expect
        g.debug_fail_member(0)
        with pytest.raises(phj.PhjError) as e:
            g.join(p)
        assert e.value.code == PHJ_ERR_STATE
        assert g.join(p).matches == expect
        assert g.join(p).matches == expect


@pytest.mark.parametrize("name,p", PARAMS[:2], ids=[a for a, _ in PARAMS[:2]])
@pytest.mark.parametrize("world", [2, 3])
def test_member_pack_matches_protocol(world, name, p):
    """The library's own exchange blocks (the device pack of each member,
    phj_debug_exchange_block) against the protocol's restatement
    (tests/exchange_proto.py, the same pack tests/test_distributed.py runs over
    gloo): layout, bounds and each segment's codes."""
    import exchange_proto as X
    R, S = O.generate_tables(300_007, 2_000_003, 1.05, 13, threads=4)
    R[:, 0] = R[:, 0] * 7919 - 3   # spread keys: no structure in the codes
    nR = R.shape[0]
    with phj.Context(devices=[0] * world, flags=phj.CTX_LOCAL) as g:
        g.upload(phj.SIDE_BUILD, R)
        g.upload(phj.SIDE_PROBE, S)
        g.join(p)
        nseg, _ = X.geometry(p, nR)
        maxn = max(hi - lo for lo, hi in (shard_range(nR, r, world) for r in range(world)))
        ce, be = phj.exchange_layout(maxn, nseg)
        for r in range(world):
            lo, hi = shard_range(nR, r, world)
            want = X.pack(R[lo:hi], p, nR, ce, be)
            got = g.debug_exchange_block(r, be)
            assert X.same_block(got, want, nseg, ce), (r, name)
