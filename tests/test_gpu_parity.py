"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar: bit-exact — hash values, the partitioned relation layout (keys,
payloads, partition bounds) and the matched-key counts.
"""
import os
import numpy as np
import pytest

import partitionedhashjoin_amd as phj
from oracle import oracle as O
from hashinv import preimage, table_edge_codes

pytestmark = pytest.mark.gpu

I64_MIN = -(2 ** 63)
I64_MAX = 2 ** 63 - 1
SEED = 0x1234_5678_9ABC_DEF1


def _hash_kind(h):
    return O.HASH_MURMUR3 if h == phj.HASH_MURMUR3 else O.HASH_XXH3


def test_device_hash_matches_oracle(ctx):
    rng = np.random.default_rng(7)
    keys = np.concatenate([rng.integers(I64_MIN, I64_MAX, 4000, dtype=np.int64, endpoint=True),
                           np.array([0, 1, -1, I64_MIN, I64_MAX, 2 ** 32, -(2 ** 32)], dtype=np.int64)])
    for kind in (phj.HASH_XXH3, phj.HASH_MURMUR3):
        for seed in (0, 1, SEED, 2 ** 64 - 1):
            dev = ctx.hash_keys(kind, seed, keys)
            ref = O.hash_keys(_hash_kind(kind), keys, seed)
            assert np.array_equal(dev, ref), (kind, seed)


PART_CASES = [
    # (radix bits, num_partitions, hash)
    ((4, 0), 0, phj.HASH_MURMUR3),
    ((8, 8), 0, phj.HASH_MURMUR3),
    ((3, 5), 0, phj.HASH_XXH3),
    ((11, 0), 0, phj.HASH_XXH3),
    ((11, 11), 0, phj.HASH_MURMUR3),
    ((1, 0), 32, phj.HASH_XXH3),      # reference default -p 32: hash % 32
    ((1, 0), 1000, phj.HASH_XXH3),    # non power of two
    ((1, 0), 5000, phj.HASH_XXH3),    # > 2048: two passes of hash % P
    ((1, 0), 1, phj.HASH_XXH3),
]


@pytest.mark.parametrize("bits,nparts,hk", PART_CASES)
@pytest.mark.parametrize("n", [0, 1, 2047, 2048, 2049, 100_003])
def test_partition_layout_matches_oracle(ctx, chunk_ctx, bits, nparts, hk, n):
    rng = np.random.default_rng(n + 17 * nparts + bits[0])
    rel = np.stack([rng.integers(-50_000, 50_000, n, dtype=np.int64),
                    np.arange(n, dtype=np.int64)], axis=1)
    if nparts:
        P, radix = nparts, False
    else:
        P, radix = 1 << (bits[0] + bits[1]), True
    out, obounds = O.partition(rel, P, radix, _hash_kind(hk), SEED, workers=3)
    ctx.upload(phj.SIDE_PROBE, rel)
    chunk_ctx.upload(phj.SIDE_PROBE, rel)
    for c, stable in ((ctx, True), (ctx, False), (chunk_ctx, False)):
        p = phj.radix_params(bits=bits, num_partitions=nparts, hash=hk, seed=SEED, stable=stable)
        v = c.partition(phj.SIDE_PROBE, p)
        keys, pays, bounds = c.download_partitioned(v)
        assert v.num_partitions >= P
        assert np.array_equal(bounds[:P + 1].astype(np.uint64), obounds)
        assert np.all(bounds[P:] == n)
        if stable:   # the reference's exact layout
            assert np.array_equal(keys, out[:, 0])
            assert np.array_equal(pays, out[:, 1])
        else:        # same tuples in every partition, order inside a partition unspecified
            assert_same_partitions(keys, pays, bounds, out, obounds)


def assert_same_partitions(keys, pays, bounds, out, obounds):
    """Partition by partition, the device tuples are a permutation of the
    oracle's (the unordered layout of include/phj.h PHJ_PART_STABLE)."""
    sizes = np.diff(np.asarray(obounds, dtype=np.int64))
    pid = np.repeat(np.arange(len(sizes)), sizes)
    got = np.lexsort((pays, keys, pid))
    ref = np.lexsort((out[:, 1], out[:, 0], pid))
    assert np.array_equal(keys[got], out[ref, 0])
    assert np.array_equal(pays[got], out[ref, 1])


@pytest.mark.parametrize("n", [4096 * 3, 1_000_003])
def test_unordered_partition_under_skew(chunk_ctx, n):
    ctx = chunk_ctx
    # chunked pass 1: a hot key fills many chunks of one digit's chain, runs
    # straddle chunk boundaries, and every other digit ends in a partial chunk
    rng = np.random.default_rng(n)
    keys = rng.integers(-(1 << 40), 1 << 40, n, dtype=np.int64)
    keys[rng.random(n) < 0.4] = 7
    rel = np.stack([keys, np.arange(n, dtype=np.int64)], axis=1)
    ctx.upload(phj.SIDE_PROBE, rel)
    for bits, hk in (((8, 8), phj.HASH_MURMUR3), ((4, 9), phj.HASH_XXH3), ((9, 2), phj.HASH_XXH3)):
        out, ob = O.partition(rel, 1 << (bits[0] + bits[1]), True, _hash_kind(hk), SEED, workers=2)
        for _ in range(2):   # a second pass reuses the chunk table (next generation)
            v = ctx.partition(phj.SIDE_PROBE, phj.radix_params(bits, hash=hk, seed=SEED))
            k, pay, b = ctx.download_partitioned(v)
            assert np.array_equal(b[:len(ob)].astype(np.uint64), ob)
            assert_same_partitions(k, pay, b, out, ob)


def _gpu_count(ctx, R, S, params):
    ctx.upload(phj.SIDE_BUILD, O.as_relation(R))
    ctx.upload(phj.SIDE_PROBE, O.as_relation(S))
    return ctx.join(params).matches


ALL_PARAMS = [
    ("np-xxh3", phj.nopart_params(hash=phj.HASH_XXH3, seed=SEED)),
    ("np-murmur", phj.nopart_params(hash=phj.HASH_MURMUR3, seed=3, table_ratio=1.0)),
    ("radix-8+8-murmur", phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED)),
    ("radix-4-xxh3", phj.radix_params((4, 0), hash=phj.HASH_XXH3, seed=5)),
    ("radix-11+11", phj.radix_params((11, 11), hash=phj.HASH_MURMUR3, seed=9)),
    ("radix-mod32", phj.radix_params(num_partitions=32, hash=phj.HASH_XXH3, seed=SEED)),
    ("radix-mod1", phj.radix_params(num_partitions=1, hash=phj.HASH_XXH3, seed=1)),
    ("radix-mod5000", phj.radix_params(num_partitions=5000, hash=phj.HASH_XXH3, seed=2)),
    # bucket-chained tables, the reference's SeparateChainingHashTable (PHJ_TABLE_CHAINED)
    ("radix-8+8-chained", phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED, chained=True)),
    ("radix-mod1000-chained", phj.radix_params(num_partitions=1000, hash=phj.HASH_XXH3, seed=4, chained=True)),
]


@pytest.mark.parametrize("name,params", ALL_PARAMS, ids=[a for a, _ in ALL_PARAMS])
def test_adversarial_semijoin(ctx, name, params):
    # duplicates in R, misses, 0/-1/INT64_MIN/INT64_MAX; semi-join count 8
    R = [1, 1, 2, 0, -1, I64_MIN, I64_MAX]
    S = [1, 2, 3, 0, -1, -1, I64_MIN, I64_MAX, 5, 1]
    assert _gpu_count(ctx, R, S, params) == 8 == O.join_nopart(R, S).matches


@pytest.mark.parametrize("name,params", ALL_PARAMS, ids=[a for a, _ in ALL_PARAMS])
def test_random_relations(ctx, name, params):
    rng = np.random.default_rng(11)
    R = rng.integers(-3000, 3000, 20_000, dtype=np.int64)   # heavy duplicates
    S = rng.integers(-6000, 6000, 150_000, dtype=np.int64)  # ~half misses
    expect = O.semijoin_count(R, S)
    assert O.join_radix(R, S, P=64).matches == expect
    assert _gpu_count(ctx, R, S, params) == expect


@pytest.mark.parametrize("name,params", ALL_PARAMS, ids=[a for a, _ in ALL_PARAMS])
def test_extreme_keys(ctx, name, params):
    rng = np.random.default_rng(5)
    R = rng.integers(I64_MIN, I64_MAX, 5000, dtype=np.int64, endpoint=True)
    S = np.concatenate([R[::3], rng.integers(I64_MIN, I64_MAX, 5000, dtype=np.int64,
                                             endpoint=True), [I64_MIN, I64_MAX, 0]])
    rng.shuffle(S)
    assert _gpu_count(ctx, R, S, params) == O.semijoin_count(R, S)


def edge_keys(params):
    """Keys whose codes are the code tables' empty values and their bucket
    mates (hashinv.table_edge_codes) under the plan's hash and seed."""
    mur = params.hash == phj.HASH_MURMUR3
    return np.array([preimage(mur, c, params.hash_seed) for c in table_edge_codes(params.num_partitions)],
                    dtype=np.int64)


@pytest.mark.parametrize("name,params", ALL_PARAMS, ids=[a for a, _ in ALL_PARAMS])
def test_empty_value_preimages(ctx, name, params):
    # the code tables mark an empty slot with E_p, a code of
    # another partition (csrc/phj_table.h); the reference reserves no key
    # (src/HashTables/LinearProbing.hpp:79-82). Keys hashing to 0, 1, 2^40 and
    # to their partition's home bucket, planted in S only, must all miss (no
    # false positive); planted in R, they must all be found and must not cut
    # other keys' walks short (no false negative). |R| = 20000 sub-partitions
    # h % 1 at bit 40 (where code 1 lies in partition 0) and sends every
    # 2-pass plan through the on-chip probe.
    pre = edge_keys(params)
    base = np.arange(1, 20_001, dtype=np.int64)
    base = base[~np.isin(base, pre)]
    S = np.concatenate([pre, base[::3], pre[::-1], -base[:500]])
    exp_s = O.semijoin_count(base, S)
    assert exp_s == base[::3].shape[0]
    assert _gpu_count(ctx, base, S, params) == exp_s
    R = np.concatenate([base, pre, pre[:5]])
    exp_r = O.semijoin_count(R, S)
    assert exp_r == exp_s + 2 * pre.shape[0]
    assert _gpu_count(ctx, R, S, params) == exp_r
    # every planted key alone against R holding them all
    assert _gpu_count(ctx, R, pre, params) == pre.shape[0]


def test_code_one_under_mod1_is_not_empty(ctx):
    # the concrete round-3 false positive: under XXH3 seed 1 the key below has
    # code 1, which lies in partition 0 of h % 1 split at bit 40
    p = phj.radix_params(num_partitions=1, hash=phj.HASH_XXH3, seed=1)
    R = np.arange(1, 20_001, dtype=np.int64)
    assert _gpu_count(ctx, R, [-6993838658721465140], p) == 0
    assert _gpu_count(ctx, np.append(R, -6993838658721465140), [-6993838658721465140, 5], p) == 2


@pytest.mark.parametrize("name,params", ALL_PARAMS, ids=[a for a, _ in ALL_PARAMS])
def test_all_keys_equal(ctx, name, params):
    # one hot key: every tuple of both relations lands in one partition/bucket chain
    R = np.full(3000, 42, dtype=np.int64)
    S = np.concatenate([np.full(50_000, 42, dtype=np.int64), np.arange(100, dtype=np.int64)])
    assert _gpu_count(ctx, R, S, params) == 50_000 + 1


@pytest.mark.parametrize("name,params", ALL_PARAMS, ids=[a for a, _ in ALL_PARAMS])
def test_empty_probe(ctx, name, params):
    assert _gpu_count(ctx, [1, 2, 3], np.zeros(0, dtype=np.int64), params) == 0


def test_empty_build_radix_is_zero(ctx):
    assert _gpu_count(ctx, np.zeros(0, dtype=np.int64), [1, 2, 3],
                      phj.radix_params((8, 8))) == 0


def test_empty_build_nopartitioning_raises(ctx):
    # LinearProbing.hpp:295-299: numberOfObjects must be greater than zero
    with pytest.raises(phj.PhjError, match="numberOfObjects"):
        _gpu_count(ctx, np.zeros(0, dtype=np.int64), [1, 2, 3], phj.nopart_params())


@pytest.mark.parametrize("alpha", [1.05, 1.25])
@pytest.mark.parametrize("name,params", ALL_PARAMS[:6], ids=[a for a, _ in ALL_PARAMS[:6]])
def test_seeded_zipf_workload(ctx, name, params, alpha):
    # generateTables (main.cpp:35-79) at 1e5 x 2e6 with a seed; count == |S|
    R, S = O.generate_tables(100_000, 2_000_000, alpha, seed=77)
    ref = O.join_radix(R, S, P=1024, workers=4)
    assert ref.matches == S.shape[0]
    assert _gpu_count(ctx, R, S, params) == ref.matches


def test_reference_partition_count_matches_gpu_P1024(ctx):
    # the reference's best published configuration (-p 1024, XXH3) on the GPU
    R, S = O.generate_tables(50_000, 800_000, 1.05, seed=3)
    S[::7, 0] = -S[::7, 0]   # knock out a seventh of the probe keys
    exp = O.join_radix(R, S, P=1024, part_seed=SEED, table_seed=4).matches
    assert exp == O.semijoin_count(R, S)
    assert _gpu_count(ctx, R, S, phj.radix_params(num_partitions=1024, hash=phj.HASH_XXH3,
                                                  seed=SEED)) == exp


def test_join_partitioned_multi_segment(ctx):
    # multi-GPU building block: R split in 3 shards partitioned by separate
    # contexts, joined as 3 build segments against one partitioned S
    rng = np.random.default_rng(3)
    R = np.stack([rng.integers(0, 200_000, 60_000, dtype=np.int64),
                  np.arange(60_000, dtype=np.int64)], axis=1)
    S = np.stack([rng.integers(0, 400_000, 500_000, dtype=np.int64),
                  np.arange(500_000, dtype=np.int64)], axis=1)
    p = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED)
    shards = np.array_split(R, 3)
    ctxs = [phj.Context(0) for _ in shards]
    try:
        segs = []
        for c, sh in zip(ctxs, shards):
            c.upload(phj.SIDE_BUILD, sh)
            segs.append(c.partition(phj.SIDE_BUILD, p))
        for c in ctxs:
            c.synchronize()
        ctx.upload(phj.SIDE_PROBE, S)
        ctx.partition(phj.SIDE_PROBE, p)
        r = ctx.join_partitioned(p, segs)
        assert r.matches == O.semijoin_count(R, S)
        # asynchronous form: the count lands in device memory, stream-ordered
        import torch
        cnt = torch.full((1,), -1, dtype=torch.int64, device="cuda:0")
        torch.cuda.synchronize()
        ctx.join_partitioned_async(p, segs, cnt.data_ptr())
        ctx.synchronize()
        assert int(cnt.item()) == r.matches
        t = ctx.timers_report().timers()
        assert {"build", "probe"} <= {name for name, _, _ in t}
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("fused", ["1", "0"])
def test_hot_build_partition_over_segments(fused, monkeypatch):
    # one build key repeated 5000 times (its partition exceeds one 512-key LDS
    # table round of the fused join) next to ordinary keys, split over 4 build
    # segments; S holds the hot key, ordinary hits and misses
    monkeypatch.setenv("PHJ_FUSED", fused)
    rng = np.random.default_rng(17)
    hot = 123_456_789
    rk = np.concatenate([np.full(5000, hot, dtype=np.int64), rng.integers(0, 300_000, 40_000, dtype=np.int64)])
    rng.shuffle(rk)
    R = np.stack([rk, np.arange(rk.size, dtype=np.int64)], axis=1)
    sk = np.concatenate([np.full(7000, hot, dtype=np.int64), rng.integers(0, 600_000, 300_000, dtype=np.int64)])
    rng.shuffle(sk)
    S = np.stack([sk, np.arange(sk.size, dtype=np.int64)], axis=1)
    p = phj.radix_params((8, 8), hash=phj.HASH_XXH3, seed=SEED)
    ctxs = [phj.Context(0) for _ in range(5)]
    try:
        segs = []
        for c, sh in zip(ctxs[1:], np.array_split(R, 4)):
            c.upload(phj.SIDE_BUILD, sh)
            segs.append(c.partition(phj.SIDE_BUILD, p))
            c.synchronize()
        main = ctxs[0]
        main.upload(phj.SIDE_PROBE, S)
        main.partition(phj.SIDE_PROBE, p)
        r = main.join_partitioned(p, segs)
        assert r.matches == O.semijoin_count(R, S)
        assert r.build_ms >= 0 and r.probe_ms >= 0
        # and the single-call join over the whole relation
        main.upload(phj.SIDE_BUILD, R)
        assert main.join(p).matches == r.matches
    finally:
        for c in ctxs:
            c.close()


def test_partitioned_download_to_device_is_stream_ordered(ctx):
    import torch
    rng = np.random.default_rng(5)
    rel = np.stack([rng.integers(0, 1 << 40, 70_001, dtype=np.int64), np.arange(70_001, dtype=np.int64)], axis=1)
    p = phj.radix_params((6, 5), hash=phj.HASH_XXH3, seed=SEED)
    ctx.upload(phj.SIDE_PROBE, rel)
    v = ctx.partition(phj.SIDE_PROBE, p)
    hk, hp, hb = ctx.download_partitioned(v)
    dk = torch.zeros(v.n, dtype=torch.int64, device="cuda:0")
    dp = torch.zeros(v.n, dtype=torch.int64, device="cuda:0")
    db = torch.zeros(v.num_partitions + 1, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    import ctypes as C
    ctx._check(ctx._L.phj_partitioned_download(ctx._h, C.byref(v), C.c_void_p(dk.data_ptr()),
                                               C.c_void_p(dp.data_ptr()), C.c_void_p(db.data_ptr())))
    ctx.synchronize()
    assert np.array_equal(dk.cpu().numpy(), hk)
    assert np.array_equal(dp.cpu().numpy(), hp)
    assert np.array_equal(db.cpu().numpy().view(np.uint32), hb)


@pytest.mark.parametrize("alpha", [1.05, 1.25, 0.995])
def test_gpu_generators(ctx, alpha):
    ctx.generate_sequential(phj.SIDE_BUILD, 10_000, 1)
    assert np.array_equal(ctx.download(phj.SIDE_BUILD), O.fill_sequential(10_000, 1))
    # the device Zipf generator evaluates glibc's pow bit for bit (csrc/phj_pow.h):
    # every sample of >= 1M equals the host generator's (the reference's own
    # Zipf.cpp, test_host_generators_match_reference_outputs), so the bench's
    # device-generated inputs are the reference generator's inputs
    n = 4096 * 300 + 5
    ctx.generate_zipf(phj.SIDE_PROBE, n, alpha, 1, 10_000_000, 99)
    dev = ctx.download(phj.SIDE_PROBE)
    host = O.fill_zipf(n, alpha, 1, 10_000_000, 99)
    assert np.array_equal(dev, host)
    assert ctx.count_in_range(phj.SIDE_PROBE, 1, 10_000_000) == n


def test_large_generated_workload_property(ctx):
    # size-independent property at 2M x 40M: every S key lies in [1, |R|], so the
    # semi-join count is |S|, and all algorithms agree.
    nR, nS = 2_000_000, 40_000_000
    ctx.generate_sequential(phj.SIDE_BUILD, nR, 1)
    ctx.generate_zipf(phj.SIDE_PROBE, nS, 1.05, 1, nR, 5)
    inrange = ctx.count_in_range(phj.SIDE_PROBE, 1, nR)
    assert inrange == nS
    for p in (phj.radix_params((8, 8)), phj.radix_params((11, 0), hash=phj.HASH_XXH3),
              phj.nopart_params()):
        assert ctx.join(p).matches == inrange


@pytest.mark.parametrize("params", [phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED),
                                    phj.radix_params(num_partitions=32, hash=phj.HASH_XXH3, seed=SEED),
                                    phj.nopart_params(hash=phj.HASH_XXH3, seed=SEED)])
def test_prepare_then_join(params):
    # phj_prepare allocates the workspace for the bound relations; the join that
    # follows is unchanged (fresh context: nothing was allocated before)
    R, S = O.generate_tables(50_000, 600_001, 1.05, 31, threads=4)
    with phj.Context(0) as c:
        c.upload(phj.SIDE_BUILD, R)
        c.upload(phj.SIDE_PROBE, S)
        c.prepare(params)
        assert c.join(params).matches == O.semijoin_count(R, S)


@pytest.mark.parametrize("params,env", [
    (phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED), {}),                       # fused LDS join
    (phj.radix_params(num_partitions=2, hash=phj.HASH_XXH3, seed=SEED), {}),                # bucket tables
    (phj.radix_params(num_partitions=64, hash=phj.HASH_XXH3, seed=SEED), {"PHJ_PTAB": "0"}),  # CSR tables
])
def test_key_only_build_segments(params, env, monkeypatch):
    # the multi-GPU exchange ships build keys only (payloads NULL in every segment)
    import ctypes
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(23)
    R = np.stack([rng.integers(0, 400_000, 150_000, dtype=np.int64), np.arange(150_000, dtype=np.int64)], axis=1)
    S = np.stack([rng.integers(0, 800_000, 700_000, dtype=np.int64), np.arange(700_000, dtype=np.int64)], axis=1)
    ctxs = [phj.Context(0) for _ in range(4)]
    try:
        segs = []
        for c, sh in zip(ctxs[1:], np.array_split(R, 3)):
            c.upload(phj.SIDE_BUILD, sh)
            v = c.partition(phj.SIDE_BUILD, params)
            c.synchronize()
            v.payloads = None
            segs.append(v)
        main = ctxs[0]
        main.upload(phj.SIDE_PROBE, S)
        main.partition(phj.SIDE_PROBE, params)
        assert main.join_partitioned(params, segs).matches == O.semijoin_count(R, S)
        # mixing key-only and full segments is rejected
        segs[0].payloads = ctypes.c_void_p(segs[1].keys).value
        with pytest.raises(phj.PhjError):
            main.join_partitioned(params, segs)
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("ratio", [0.0, 1.0])
def test_nopart_hot_build_key_overflow(ctx, ratio):
    """A build key repeated 40K times: in the count's region code table it
    fills one region's table far past its LDS slice (k_ht_fill's in-place
    path); in the materialised join's 64-B bucket table, built region by
    region in LDS, it spills through the overflow list into the next regions
    and the probe walks the same way. Both agree with the oracle."""
    rng = np.random.default_rng(5)
    R = np.concatenate([np.full(40_000, 7, dtype=np.int64),
                        rng.integers(-200_000, 200_000, 300_000, dtype=np.int64)])
    rng.shuffle(R)
    S = rng.integers(-400_000, 400_000, 2_000_000, dtype=np.int64)
    S[::50] = 7
    expect = O.semijoin_count(O.as_relation(R), O.as_relation(S))
    ctx.upload(phj.SIDE_BUILD, O.as_relation(R))
    ctx.upload(phj.SIDE_PROBE, O.as_relation(S))
    for hk in (phj.HASH_XXH3, phj.HASH_MURMUR3):
        p = phj.nopart_params(hash=hk, seed=SEED, table_ratio=ratio)
        assert ctx.join(p).matches == expect
        assert ctx.join_materialize(p).matches == expect


# ---- the LDS join (csrc/phj_cluster.h): cluster tables in LDS, big clusters in HBM ----

def _cluster_ctx(monkeypatch, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    return phj.Context(0)


@pytest.mark.parametrize("env", [{}, {"PHJ_CL_CAP": "8192"}, {"PHJ_CL_BITS": "11"}, {"PHJ_CL_BITS": "9", "PHJ_CL_CAP": "8192"}],
                         ids=["default", "cap8192", "bits11", "bits9-cap8192"])
@pytest.mark.parametrize("name,params", [a for a in ALL_PARAMS if a[0].startswith("radix") and "chained" not in a[0]],
                         ids=[a[0] for a in ALL_PARAMS if a[0].startswith("radix") and "chained" not in a[0]])
def test_cluster_tables_lds_and_hbm(monkeypatch, env, name, params):
    """A build side whose clusters fit the LDS table except one: a hot key
    repeated beyond the LDS limit (its cluster's table goes to HBM,
    k_cluster_big_fill), many keys with few repeats, the extremes and the
    empty-value preimages of the plan; probes hit the hot cluster, the LDS
    clusters and miss. Counted against the oracle's sort-and-search."""
    c = _cluster_ctx(monkeypatch, **env)
    try:
        rng = np.random.default_rng(len(name) * 131 + len(env))
        hk = params.hash
        pre = [preimage(hk == phj.HASH_MURMUR3, x, params.hash_seed) for x in table_edge_codes(0)]
        R = np.concatenate([np.full(20_000, 777, dtype=np.int64),
                            rng.integers(-400_000, 400_000, 180_000, dtype=np.int64),
                            np.array([0, -1, I64_MIN, I64_MAX] + pre[::2], dtype=np.int64)])
        S = np.concatenate([np.full(30_000, 777, dtype=np.int64),
                            rng.integers(-800_000, 800_000, 600_000, dtype=np.int64),
                            np.array([0, -1, I64_MIN, I64_MAX, 5] + pre, dtype=np.int64)])
        rng.shuffle(R)
        rng.shuffle(S)
        expect = O.semijoin_count_keys(R, S)
        assert _gpu_count(c, R, S, params) == expect
        assert c.join(params).matches == expect   # the buffers reused
    finally:
        c.close()


@pytest.mark.parametrize("env", [{}, {"PHJ_R_CHUNK": "0"}], ids=["tiles", "stable"])
def test_cluster_tile_mode_runs(monkeypatch, env):
    """R through the chunked code pass (tile mode, the one-device default):
    a cluster's R codes are read through its pass-1 tiles. Here one key
    repeated 150K times makes its cluster span more tiles than a build reads
    at once (8 shards x ~5 chunks: the HBM table, read tile by tile), a second
    cluster sits just under the LDS limit in several runs, and R is small
    enough elsewhere for one-tile clusters. Counted against the oracle."""
    c = _cluster_ctx(monkeypatch, **env)
    try:
        params = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED)
        rng = np.random.default_rng(77)
        R = np.concatenate([np.full(150_000, 4242, dtype=np.int64), np.full(11_000, -99, dtype=np.int64),
                            rng.integers(-3_000_000, 3_000_000, 900_000, dtype=np.int64)])
        S = np.concatenate([np.full(40_000, 4242, dtype=np.int64), np.full(7_000, -99, dtype=np.int64),
                            rng.integers(-6_000_000, 6_000_000, 1_500_000, dtype=np.int64)])
        rng.shuffle(R)
        rng.shuffle(S)
        expect = O.semijoin_count_keys(R, S)
        assert _gpu_count(c, R, S, params) == expect
        assert c.join(params).matches == expect
    finally:
        c.close()


@pytest.mark.parametrize("env", [{}, {"PHJ_R_CHUNK": "0"}, {"PHJ_COUNT_PIN": "0"}], ids=["tiles", "stable", "copy"])
def test_cluster_many_big(monkeypatch, env):
    """Hundreds of clusters above the LDS limit (300 hot keys, 13K copies
    each, beside 1M distinct keys): each of k_cluster_probe_big's workgroups
    finds several big clusters in its share and probes them in turn; its last
    workgroup writes the count to the host (PHJ_COUNT_PIN=0: the count is
    copied back). Counted against the oracle."""
    c = _cluster_ctx(monkeypatch, **env)
    try:
        params = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED)
        rng = np.random.default_rng(91)
        hot = rng.choice(np.arange(-10_000_000, 10_000_000, dtype=np.int64), 300, replace=False)
        R = np.concatenate([np.repeat(hot, 13_000), rng.integers(-20_000_000, 20_000_000, 1_000_000, dtype=np.int64)])
        S = np.concatenate([hot[::2], rng.integers(-40_000_000, 40_000_000, 2_000_000, dtype=np.int64)])
        rng.shuffle(R)
        rng.shuffle(S)
        expect = O.semijoin_count_keys(R, S)
        assert _gpu_count(c, R, S, params) == expect
        assert c.join(params).matches == expect
    finally:
        c.close()


def test_deferred_timers(ctx):
    """PHJ_DEFER_TIMERS: the join's result carries its count but no timers;
    the context keeps them, and timers_report returns their sums over the
    deferred joins (then a normal join reports its own again)."""
    ctx.generate_sequential(phj.SIDE_BUILD, 1_000_000, 1)
    ctx.generate_zipf(phj.SIDE_PROBE, 3_000_000, 1.05, 1, 1_000_000, 9)
    p = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED)
    one = ctx.join(p)
    single = {name: ms for name, ms, _ in one.timers()}
    assert one.matches == 3_000_000 and single
    q = type(p).from_buffer_copy(p)
    q.flags = p.flags | phj.DEFER_TIMERS
    ctx.timers_report()
    for _ in range(3):
        r = ctx.join(q)
        assert r.matches == 3_000_000
        assert list(r.timers()) == [] and r.total_ms == 0
    summed = {name: ms for name, ms, _ in ctx.timers_report().timers()}
    assert set(summed) == set(single)
    for name in ("S.p1.scatter", "probe"):
        assert summed[name] > 1.5 * single[name]   # three joins' worth
    # PHJ_LEAN_TIMERS: the build side's pass-1 timers are not recorded,
    # build.big is listed at zero; back-to-back joins reuse S's chunk state
    # cleared by the previous join's last workgroup
    q.flags = p.flags | phj.DEFER_TIMERS | phj.LEAN_TIMERS
    for _ in range(3):
        assert ctx.join(q).matches == 3_000_000
    lean = {name: ms for name, ms, _ in ctx.timers_report().timers()}
    assert not [n for n in lean if n.startswith("R.")] and lean["build.big"] == 0
    assert {"S.p1.scatter", "build", "probe"} <= set(lean) and lean["S.p1.scatter"] > 1.5 * single["S.p1.scatter"]
    assert ctx.join(p).timers()


def test_cleared_chunk_state_between_calls(ctx):
    """The LDS join's last workgroup clears S's chunk state for the next
    join's pass 1 (no memset): deferred and plain joins interleaved with an
    unordered partition of S stay exact, the partition matches the oracle's
    (the stale-table failure, after which the state is not cleared:
    test_gpu_chunk_guard.py)."""
    R, S = O.generate_tables(200_000, 1_500_003, 1.05, 5, threads=4)
    S[::5, 0] += 200_000
    expect = O.semijoin_count(R, S)
    ctx.upload(phj.SIDE_BUILD, R)
    ctx.upload(phj.SIDE_PROBE, S)
    p = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED)
    q = type(p).from_buffer_copy(p)
    q.flags = p.flags | phj.DEFER_TIMERS | phj.LEAN_TIMERS
    for params in (q, q, p, q):
        assert ctx.join(params).matches == expect
    u = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED, stable=False)
    out, ob = O.partition(S, 1 << 16, True, O.HASH_MURMUR3, SEED, workers=2)
    k, pay, bounds = ctx.download_partitioned(ctx.partition(phj.SIDE_PROBE, u))
    assert_same_partitions(k, pay, bounds, out, ob)
    for params in (q, p):
        assert ctx.join(params).matches == expect
    ctx.timers_report()


def test_cluster_path_is_default_for_c2_shape(ctx):
    """10M-scale build side at 8+8 radix bits: the join's pass 1 is the LDS
    join's 1024 clusters (the probe-side pass-1 hook reports its digits)."""
    nR, nS = 10_000_000, 4_000_000
    ctx.generate_sequential(phj.SIDE_BUILD, nR, 1)
    ctx.generate_zipf(phj.SIDE_PROBE, nS, 1.05, 1, nR, 5)
    p = phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED)
    out, b1, codes = ctx.probe_pass1(p)
    assert codes and b1.shape[0] == 1025
    assert ctx.join(p).matches == nS
