"""Hash codes stand in for keys in the counting join (csrc/phj_hash.h kHashed).

The keys-only pass 1 writes h(k) instead of k and the code tables store h(r),
so the probe compares codes. That counts the key matches of
/root/reference/src/RadixCluster/HashJoin.hpp:295-301 exactly iff h is a
bijection of the 64-bit keys. Here both hashes are inverted step by step
(against the oracle's forward hashes, which are pinned to xxhash / the
canonical fmix64 constants) on random and extreme keys and several seeds:
a left inverse on every sample is that bijection, observed.
"""
import numpy as np
import pytest

from oracle import oracle as O
from hashinv import murmur3_inverse, preimage, table_edge_codes, xxh3_inverse

M64 = (1 << 64) - 1
SEEDS = [0, 1, 0x0BAD_5EED_0BAD_5EED, 0xFFFF_FFFF_FFFF_FFFF]


def _keys():
    rng = np.random.default_rng(7)
    k = [0, 1, 2, -1, 2**63 - 1, -(2**63), 2**32, 2**32 - 1, -(2**32), 10_000_000]
    k += [int(v) for v in rng.integers(-(2**63), 2**63 - 1, 150, dtype=np.int64)]
    k += list(range(1, 40))
    return k


@pytest.mark.parametrize("seed", SEEDS)
def test_murmur3_is_a_bijection(seed):
    for k in _keys():
        u = k & M64
        h = O.murmur3(u, seed) & M64
        assert murmur3_inverse(h, seed) == u


@pytest.mark.parametrize("seed", SEEDS)
def test_xxh3_is_a_bijection(seed):
    for k in _keys()[:60]:
        u = k & M64
        h = O.xxh3(u, seed) & M64
        assert xxh3_inverse(h, seed) == u


def test_codes_preserve_the_join_count():
    # counting over codes == counting over keys, for both hashes
    rng = np.random.default_rng(3)
    r = rng.integers(-5000, 5000, 3000, dtype=np.int64)
    s = rng.integers(-9000, 9000, 20000, dtype=np.int64)
    s[::5] = r[: len(s[::5]) % len(r) or 1][0]
    expect = O.semijoin_count_keys(r, s)
    for kind in (O.HASH_MURMUR3, O.HASH_XXH3):
        hr = O.hash_keys(kind, r, 11).view(np.int64)
        hs = O.hash_keys(kind, s, 11).view(np.int64)
        assert O.semijoin_count_keys(hr, hs) == expect


@pytest.mark.parametrize("nparts", [0, 1, 32, 1000, 5000])
def test_edge_code_preimages(nparts):
    # the keys the GPU parity tests plant (test_gpu_parity.py
    # test_empty_value_preimages): each hashes to its chosen code
    codes = table_edge_codes(nparts)
    assert {0, 1, 1 << 40} <= set(codes)
    for kind, mur in ((O.HASH_MURMUR3, True), (O.HASH_XXH3, False)):
        for seed in (1, 0x1234_5678_9ABC_DEF1):
            keys = np.array([preimage(mur, c, seed) for c in codes], dtype=np.int64)
            assert np.array_equal(O.hash_keys(kind, keys, seed), np.array(codes, dtype=np.uint64))


def test_known_code_one_key():
    # under XXH3 seed 1 this key's code is 1, which the
    # round-3 tables used as partition 0's empty value under h % 1
    k = -6993838658721465140
    assert preimage(False, 1, 1) == k
    assert int(O.hash_keys(O.HASH_XXH3, np.array([k], dtype=np.int64), 1)[0]) == 1
