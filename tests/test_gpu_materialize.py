"""Materialised join (phj_join_materialize) against
a numpy restatement: one row {id, payloadA, payloadB} per probe tuple with a
matching build key (HashTable::Get returns the first build tuple found,
LinearProbing.hpp:160-180), same count as phj_join."""
import numpy as np
import pytest

import partitionedhashjoin_amd as phj
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED = 0x9E3779B97F4A7C15


def expected_rows(R, S):
    """(rows in probe order, {key: set of build payloads})."""
    payloads = {}
    for k, v in R:
        payloads.setdefault(int(k), set()).add(int(v))
    keep = np.isin(S[:, 0], R[:, 0])
    return S[keep], payloads


def check_rows(rows, R, S, ordered):
    exp, payloads = expected_rows(R, S)
    assert rows.shape == (len(exp), 3)
    if not ordered:   # radix: partition order; probe payloads are unique row ids
        rows = rows[np.argsort(rows[:, 2], kind="stable")]
        exp = exp[np.argsort(exp[:, 1], kind="stable")]
    assert np.array_equal(rows[:, 0], exp[:, 0])
    assert np.array_equal(rows[:, 2], exp[:, 1])
    # payloadA: a build payload of that key (the only one when build keys are unique)
    for k, a in zip(rows[:, 0].tolist(), rows[:, 1].tolist()):
        assert a in payloads[k]


PARAMS = [
    ("np-xxh3", phj.nopart_params(hash=phj.HASH_XXH3, seed=SEED), True),
    ("np-murmur-r1", phj.nopart_params(hash=phj.HASH_MURMUR3, seed=3, table_ratio=1.0), True),
    ("radix-8+8", phj.radix_params((8, 8), hash=phj.HASH_MURMUR3, seed=SEED), False),
    ("radix-mod1024", phj.radix_params(num_partitions=1024, hash=phj.HASH_XXH3, seed=7), False),
    ("radix-4", phj.radix_params((4, 0), hash=phj.HASH_XXH3, seed=2), False),
]


@pytest.mark.parametrize("name,params,ordered", PARAMS, ids=[p[0] for p in PARAMS])
def test_materialize_generated(ctx, name, params, ordered):
    R, S = O.generate_tables(50_000, 700_001, 1.05, 17, threads=4)
    S[::4, 0] += 60_000          # a quarter of the probe keys miss
    ctx.upload(phj.SIDE_BUILD, R)
    ctx.upload(phj.SIDE_PROBE, S)
    r = ctx.join_materialize(params)
    assert r.matches == ctx.join(params).matches == O.semijoin_count(R, S)
    check_rows(ctx.joined(), R, S, ordered)


@pytest.mark.parametrize("name,params,ordered", PARAMS, ids=[p[0] for p in PARAMS])
def test_materialize_duplicates_and_rounds(ctx, name, params, ordered):
    # 3000 copies of one build key: its partition takes many LDS rounds in the
    # radix join, its buckets overflow in NoPartitioning
    rng = np.random.default_rng(3)
    rk = np.concatenate([np.full(3000, 7, dtype=np.int64), rng.integers(-20_000, 20_000, 40_000)])
    rng.shuffle(rk)
    R = np.stack([rk, np.arange(len(rk), dtype=np.int64) + 1000], axis=1)
    sk = rng.integers(-40_000, 40_000, 300_000)
    sk[::9] = 7
    S = np.stack([sk, np.arange(len(sk), dtype=np.int64)], axis=1)
    ctx.upload(phj.SIDE_BUILD, R)
    ctx.upload(phj.SIDE_PROBE, S)
    r = ctx.join_materialize(params)
    assert r.matches == O.semijoin_count(R, S)
    check_rows(ctx.joined(), R, S, ordered)


def test_materialize_empty_probe_and_no_matches(ctx):
    R = np.stack([np.arange(1, 1001, dtype=np.int64), np.arange(1000, dtype=np.int64)], axis=1)
    ctx.upload(phj.SIDE_BUILD, R)
    for S in (np.zeros((0, 2), dtype=np.int64),
              np.stack([np.arange(5000, 9000, dtype=np.int64), np.arange(4000, dtype=np.int64)], axis=1)):
        ctx.upload(phj.SIDE_PROBE, S)
        for p in (phj.nopart_params(), phj.radix_params((8, 8))):
            assert ctx.join_materialize(p).matches == 0
            assert ctx.joined().shape == (0, 3)


def test_materialize_unique_keys_exact_payloads(ctx):
    # Sequential R (unique keys): payloadA is exactly the key's build payload
    R, S = O.generate_tables(20_000, 400_000, 1.25, 5, threads=4)
    ctx.upload(phj.SIDE_BUILD, R)
    ctx.upload(phj.SIDE_PROBE, S)
    pay = dict(zip(R[:, 0].tolist(), R[:, 1].tolist()))
    for p in (phj.nopart_params(), phj.radix_params((8, 8))):
        ctx.join_materialize(p)
        rows = ctx.joined()
        assert len(rows) == len(S)
        assert np.array_equal(rows[:, 1], np.array([pay[k] for k in rows[:, 0].tolist()], dtype=np.int64))
