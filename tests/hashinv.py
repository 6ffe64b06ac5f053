"""Inverses of the two device hashes (csrc/phj_hash.h), test infrastructure.

Both XXH3's 8-byte path and Murmur3's fmix64 are bijections of the 64-bit
keys; these step-by-step inverses prove it (tests/test_hash_codes.py) and turn
a chosen hash code into the key that has it (preimage keys planted by the GPU
parity tests: codes equal to a code table's empty value E_p, csrc/phj_table.h).
"""
import numpy as np

M64 = (1 << 64) - 1


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



def preimage(kind_is_murmur3, code, seed):
    """The int64 key whose hash code is `code` (uint64)."""
    u = (murmur3_inverse if kind_is_murmur3 else xxh3_inverse)(code & M64, seed & M64)
    return int(np.array([u], dtype=np.uint64).view(np.int64)[0])


def table_edge_codes(num_partitions):
    """Codes at the code tables' edges (csrc/phj_table.h, csrc/phj_cluster.h): 0, 1 and 2^40 (the
    empty values E_p of every plan: E_p = 0 for p != 0, E_0 = 1, or 2^40 under
    h % 1), 2, 3, 2^64 - 1, and "bucket mates" of 0, 1 and 2^40: codes of the
    same final partition and the same home bucket ((c >> 24) & mask = 0),
    c + (m t) << 50 with m = P for h % P (the residue mod P is kept while
    m t < 2^14) and m = 1 for radix bits and NoPartitioning regions (low bits
    kept). Planted in R they fill the bucket an E-coloured slot sits in, so a
    slot mistaken for empty ends other codes' walks early."""
    m = num_partitions if num_partitions > 0 else 1
    ts = [t for t in range(1, 9) if m * t < (1 << 14)]
    codes = {0, 1, 2, 3, 1 << 40, M64}
    for b in (0, 1, 1 << 40):
        for t in ts:
            codes.add(b + ((m * t) << 50))
    # the LDS join's cluster tables (csrc/phj_cluster.h): E of cluster 0 is the
    # plan's lowest power of two outside cluster 0 (2^(log2 P - k) for radix
    # bits, 2^40.. under h % P with sub-partition bits): every power of two,
    # and bucket mates of those a cluster plan can pick
    for b in range(64):
        codes.add(1 << b)
    for b in list(range(0, 17)) + [40, 41, 42]:
        for t in ts[:3]:
            codes.add((1 << b) + ((m * t) << 50))
    return sorted(c & M64 for c in codes)
