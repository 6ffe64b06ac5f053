// phj_hash.h — per-lane hash functions for gfx950 (and the host, for sizing).
//
// XXH3_64bits_withSeed over the 8 little-endian bytes of an int64 key is what
// Common::XXHasher::Hash computes (src/Common/XXHasher.hpp:19-22) before its
// `% cardinality`. For an 8-byte input xxHash takes its "len 4..8" path: one
// keyed 64-bit word, then the rrmxmx mixer. Only kSecret[8..24) enters it.
// Murmur3 is the 64-bit MurmurHash3 finalizer (fmix64) over key ^ seed.
// Both are a handful of 64-bit VALU ops per lane (v_mad_u64_u32, v_lshl*_b64).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define PHJ_HD __host__ __device__ __forceinline__
#else
#define PHJ_HD inline
#endif

namespace phj {

// kHashed: the column already holds hash codes h(k) (the keys-only pass 1 of
// the counting join writes them, its code tables store them), so hashing is
// the identity. Sound because both hashes are bijections of the 64-bit keys:
// fmix64 is xor-shifts and multiplies by odd constants; XXH3's 8-byte path is
// a half swap, an xor, x ^ rotl(x,49) ^ rotl(x,24) (the linear map
// 1 + R^49 + R^24 is a unit of GF(2)[R]/(R^64 + 1): it is 1 at R = 1), odd
// multiplies, h ^ ((h >> 35) + 8) (bits 30..63 pass through and determine the
// rest) and an xorshift. So h(r) == h(s) iff r == s, and comparing codes
// counts exactly the key matches of HashJoin.hpp:295-301. tests/test_oracle.py
// inverts both on random and extreme keys.
enum HashKind : int { kXXH3 = 0, kMurmur3 = 1, kHashed = 2 };

PHJ_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

PHJ_HD uint64_t xxh3_8(uint64_t key, uint64_t seed) {
    const uint32_t s = static_cast<uint32_t>(seed);
    const uint32_t swapped = (s >> 24) | ((s >> 8) & 0xff00u) | ((s << 8) & 0xff0000u) | (s << 24);
    seed ^= static_cast<uint64_t>(swapped) << 32;
    // (kSecret[8..16) ^ kSecret[16..24)) as little-endian words
    const uint64_t bitflip = (0x1cad21f72c81017cULL ^ 0xdb979083e96dd4deULL) - seed;
    // input64 = readLE32(in + 4) + (readLE32(in) << 32)  ==  rotate the key by 32
    const uint64_t input64 = (key >> 32) | (key << 32);
    uint64_t h = input64 ^ bitflip;
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= 0x9FB21C651E98DF25ULL;
    h ^= (h >> 35) + 8u;
    h *= 0x9FB21C651E98DF25ULL;
    return h ^ (h >> 28);
}

PHJ_HD uint64_t murmur3_fmix64(uint64_t key, uint64_t seed) {
    uint64_t k = key ^ seed;
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    return k ^ (k >> 33);
}

template <int HK>
PHJ_HD uint64_t hash64(uint64_t key, uint64_t seed) {
    if constexpr (HK == kMurmur3) {
        return murmur3_fmix64(key, seed);
    } else if constexpr (HK == kHashed) {
        (void)seed;
        return key;
    } else {
        return xxh3_8(key, seed);
    }
}

}  // namespace phj
