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

M64 = (1 << 64) - 1
SEEDS = [0, 1, 0x0BAD_5EED_0BAD_5EED, 0xFFFF_FFFF_FFFF_FFFF]


def _rotl(x, r):
    return ((x << r) | (x >> (64 - r))) & M64


def _inv_xorshift_right(y, s):
    # x ^= x >> s
    x = y
    for _ in range(64 // s + 1):
        x = y ^ (x >> s)
    return x


def _inv_mul(c):
    return pow(c, -1, 1 << 64)


def _xxh3_bitflip(seed):
    s = seed & 0xFFFFFFFF
    swapped = int.from_bytes(s.to_bytes(4, "little"), "big")
    seed ^= swapped << 32
    return ((0x1CAD21F72C81017C ^ 0xDB979083E96DD4DE) - seed) & M64


def _inv_lin(y):
    # x ^ rotl(x,49) ^ rotl(x,24) is linear over GF(2): invert by Gaussian
    # elimination on its 64 column images
    cols = []
    for i in range(64):
        e = 1 << i
        cols.append(e ^ _rotl(e, 49) ^ _rotl(e, 24))
    # solve A x = y: rows = output bits
    rows = []
    for bit in range(64):
        r = 0
        for i in range(64):
            if (cols[i] >> bit) & 1:
                r |= 1 << i
        rows.append([r, (y >> bit) & 1])
    piv = []
    rank = 0
    for col in range(64):
        sel = next((j for j in range(rank, 64) if (rows[j][0] >> col) & 1), None)
        assert sel is not None, "linear mixer not invertible"
        rows[rank], rows[sel] = rows[sel], rows[rank]
        for j in range(64):
            if j != rank and (rows[j][0] >> col) & 1:
                rows[j][0] ^= rows[rank][0]
                rows[j][1] ^= rows[rank][1]
        piv.append(col)
        rank += 1
    x = 0
    for j, col in enumerate(piv):
        x |= rows[j][1] << col
    return x


def xxh3_inverse(h, seed):
    C = 0x9FB21C651E98DF25
    x = _inv_xorshift_right(h, 28)
    x = (x * _inv_mul(C)) & M64
    # y = x ^ ((x >> 35) + 8): bits 30..63 of x pass through unchanged
    hi = x >> 35
    x = x ^ ((hi + 8) & M64)
    x = (x * _inv_mul(C)) & M64
    x = _inv_lin(x)
    x ^= _xxh3_bitflip(seed)
    return ((x >> 32) | (x << 32)) & M64


def murmur3_inverse(h, seed):
    x = _inv_xorshift_right(h, 33)
    x = (x * _inv_mul(0xC4CEB9FE1A85EC53)) & M64
    x = _inv_xorshift_right(x, 33)
    x = (x * _inv_mul(0xFF51AFD7ED558CCD)) & M64
    x = _inv_xorshift_right(x, 33)
    return x ^ seed


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
