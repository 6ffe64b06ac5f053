// phj_table.h — the counting radix join's build side and on-chip probe.
//
// The reference joins partition by partition: build a LinearProbing table on
// R_p, probe it with S_p, count the S tuples whose Get() finds a key
// (src/RadixCluster/HashJoin.hpp:267-303, Get() = first match,
// src/HashTables/LinearProbing.hpp:160-180). The count only tests key
// equality, and both hash functions are bijections of the 64-bit keys
// (phj_hash.h), so the join runs over hash codes c = h(k): equal codes <=>
// equal keys.
//
//   k_scatter_codes : R's pass 1, keys only, written as codes, contiguous per
//                     pass-1 digit d1 (k_hist + scan give the offsets)
//   k_ht_*          : R's pass 2 over every build segment (the shards of all
//                     ranks after the multi-GPU all-gather) into a scratch in
//                     final partition order p = d1 * nb2 + d2, then one wave per
//                     partition builds its table in LDS and writes it out
//   k_probe_ht      : the probe side's pass 2 on chip: a 4096-key pass-1 tile
//                     (one d1) is grouped by d2 in LDS and every key probes the
//                     table of its final partition
//
// Table of a final partition p: an open-addressed array of codes in 2-slot
// (16-B) buckets, cap = the smallest power of two >= 2 |R_p| slots (load
// <= 1/2; >= 1.5 |R_p| beyond one wave's LDS slice, ht_cap), home bucket (c >> 24) & (buckets - 1), linear probing over buckets
// with wrap-around, a bucket's slots filled in order, duplicates stored once
// (the count is a semi-join, a set test). There is no occupancy word and no
// key value is reserved: an empty slot holds E_p, a code of ANOTHER
// partition, which no code probing p can equal. Every partition function maps
// code 0 to partition 0 (q_from_hash: radix bits, h % P and sub-partitions
// alike), so E_p = 0 for p != 0, and E_0 = e1, a code the plan's partition
// function sends elsewhere (phj_capi.hip plan_empty0: the lowest power of two
// outside partition 0 -- 1 for radix bits and h % P with P >= 2, but 2^40 for
// h % 1 split into sub-partitions at bit 40, where code 1 IS in partition 0;
// a plan with one final partition has no such code and gets no code tables).
// The reference marks occupancy with a fill counter, never a key value
// (src/HashTables/LinearProbing.hpp:79-82). A probe reads one
// 16-B bucket (one cache line) and stops at a match or an empty slot; the CSR
// form needed a home slot plus, for a quarter to a half of the keys, a second
// line.
//
// Table layout: the region of d1 starts at slot 4 * Σ_g b1_g[d1] + 2 * nb2 * d1
// (closed form from the segments' pass-1 bounds, no scan: a partition's cap is
// < 3 |R_p| + 2), its partitions' tables follow in d2 order; desc[p] = {slot
// base, buckets - 1}.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "phj_hash.h"
#include "phj_partition.h"

namespace phj {

constexpr int kHtSegs = 16;             // build segments (ranks) per join
constexpr uint32_t kHtBucketShift = 24; // home bucket = (c >> 24) & (buckets - 1): clear of every partition bit

__host__ __device__ __forceinline__ uint32_t ht_cap_for(uint32_t want) {
    uint32_t c = 2;
    while (c < want) c <<= 1;
    return c;
}

constexpr uint32_t kHtLcap = 512;    // k_ht_fill: LDS table slots per wave

// Slots of a partition's table: the smallest power of two >= 2 m (load <=
// 1/2) while that fits one wave's LDS slice, else >= 1.5 m (load <= 2/3); at
// least one 2-slot bucket. Always < 4 m + 2 (the closed-form layout's bound).
// Measured (C2): load <= 1/2 cuts the probe's walks (a full home bucket
// without a match) from ~7 % to ~1-2 % of the keys, 0.86 -> 0.78 ms.
__host__ __device__ __forceinline__ uint32_t ht_cap(uint32_t m) {
    const uint32_t wide = ht_cap_for(2 * m);
    return wide <= kHtLcap ? wide : ht_cap_for(m + (m + 1) / 2);
}

// E_p: e1 (a code outside partition 0) for partition 0, else code 0
__host__ __device__ __forceinline__ uint64_t ht_empty(uint32_t p, uint64_t e1) { return p == 0 ? e1 : 0ull; }

// Rank of this lane's digit d among the tile's keys of digit d (counter row
// C): phj_partition.h agg_rank_lds.
__device__ __forceinline__ uint32_t agg_rank(uint32_t* C, uint32_t d, bool valid) { return agg_rank_lds(C, d, valid); }


// ---------------------------------------------------------------------------
// R pass 1: hash codes, contiguous per digit. One tile of T = BLOCK * ITEMS
// tuples per workgroup: keys loaded (8 B of each 16-B tuple), hashed, ranked
// by one LDS atomic per key (the order inside a partition is free), sorted by
// digit in LDS and written so consecutive lanes fill consecutive slots of each
// digit run. Offsets from k_hist's scanned histogram (hist[d * ntiles + t]).
// ---------------------------------------------------------------------------
__host__ __device__ constexpr size_t scatter_codes_lds_bytes(int T, uint32_t nb) {
    return static_cast<size_t>(T) * (8 + (nb <= 256 ? 1 : 2)) + static_cast<size_t>(nb) * 12 + 64 + 16;
}

template <int BLOCK, int ITEMS, int HK>
__global__ __launch_bounds__(BLOCK) void k_scatter_codes(PassArgs a) {
    __builtin_amdgcn_s_setprio(3);   // R's chain: issue ahead of the persistent S pass 1 sharing the SIMD
    constexpr int T = BLOCK * ITEMS;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t nb = a.nbins;
    int64_t* skey = reinterpret_cast<int64_t*>(smem);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(skey + T);   // [nb] counts, then tile-local starts
    uint32_t* gofs = cnt + nb;                                 // [nb]
    uint32_t* dstart = gofs + nb;                              // [nb]
    uint32_t* tmp = dstart + nb;                               // 16 words
    const SortedDigits sdig{tmp + 16, nb <= 256};              // [T]
    TileLoc L;
    if (!locate_tile<T>(a, tile_id(a), L)) return;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t n = L.hi - L.lo;
    for (uint32_t d = tid; d < nb; d += BLOCK) {
        cnt[d] = 0;
        gofs[d] = a.hist[static_cast<size_t>(d) * L.ntiles_s + L.tseg];
    }
    const longlong2* rel = reinterpret_cast<const longlong2*>(a.in_keys);
    int64_t code[ITEMS];
    uint32_t dig[ITEMS], rank[ITEMS];
    const uint32_t wbase = wave * 64 * ITEMS;
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const uint32_t e = wbase + i * 64 + lane;
        code[i] = e < n ? rel[L.lo + e].x : 0;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const uint32_t e = wbase + i * 64 + lane;
        const uint64_t h = hash64<HK>(static_cast<uint64_t>(code[i]), a.f.seed);
        code[i] = static_cast<int64_t>(h);
        dig[i] = static_cast<uint32_t>(q_from_hash(h, a.f) >> a.f.shift) & a.f.dmask;
        if (e < n) rank[i] = atomicAdd(&cnt[dig[i]], 1u);
    }
    __syncthreads();
    {
        const uint32_t dpt = (nb + BLOCK - 1) / BLOCK, d0 = tid * dpt;
        uint32_t local = 0;
        for (uint32_t j = 0; j < dpt; j++)
            if (d0 + j < nb) local += cnt[d0 + j];
        uint32_t tot;
        uint32_t run = block_exclusive_scan_t<BLOCK / 64>(local, tmp, tot);
        for (uint32_t j = 0; j < dpt; j++) {
            const uint32_t d = d0 + j;
            if (d < nb) {
                const uint32_t c = cnt[d];
                cnt[d] = run;
                dstart[d] = run;
                run += c;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const uint32_t e = wbase + i * 64 + lane;
        if (e < n) {
            const uint32_t pos = cnt[dig[i]] + rank[i];
            skey[pos] = code[i];
            sdig.put(pos, dig[i]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const uint32_t k = i * BLOCK + tid;
        if (k < n) {
            const uint32_t d = sdig.get(k);
            a.out_keys[gofs[d] + (k - dstart[d])] = skey[k];
        }
    }
}

// ---------------------------------------------------------------------------
// The build side. Every rank groups ITS OWN codes by final partition before
// the exchange (R pass 2 on the rank's shard only, k_ht_p2), so a build
// segment is {codes in partition order, bounds[P + 1]}. After the exchange
// only the tables are built over all segments (k_ht_fill: a workgroup stages
// the codes of kHtPpw consecutive partitions from every segment, each wave
// builds a partition's table in its LDS slice and writes it out).
// ---------------------------------------------------------------------------
constexpr uint32_t kHtPpw = 8;       // k_ht_fill: partitions per workgroup (two per wave)

// R pass 2 over one relation's pass-1 output (codes contiguous per d1).
struct HtPass2Args {
    const int64_t* codes;      // pass-1 output
    const uint32_t* hist1;     // pass 1's scanned histogram, hist1[d1 * nt1 + t]: d1's run starts at hist1[d1 * nt1]
    int64_t* out;              // codes in final partition order
    uint32_t* bounds;          // P + 1 final bounds
    uint32_t nt1, n;           // pass-1 tiles, codes
    uint32_t nb1, nb2;
    DigitFn f2;                // d2 = q_from_hash(c, f2) & f2.dmask (shift 0)
};

// R pass 2 in one launch: one workgroup per pass-1 digit d1 counts d1's codes by d2 in LDS, scans the
// counts itself (a digit's codes stay inside d1's run, so no other workgroup
// is involved) and scatters. A run of up to kHtP2Keep codes (the shard of a
// multi-GPU rank) is read once into registers, grouped in LDS and written out
// in order (whole lines); a longer run is counted, then read again and
// scattered through LDS cursors.
constexpr uint32_t kHtP2Block = 1024, kHtP2Items = 6;
constexpr uint32_t kHtP2Keep = kHtP2Block * kHtP2Items;

__host__ __device__ constexpr size_t ht_p2_lds_bytes(uint32_t nb2, bool keep) {
    return (keep ? static_cast<size_t>(kHtP2Keep) * 8 : 0) + static_cast<size_t>(nb2) * 8;
}

template <bool KEEP>
__global__ __launch_bounds__(kHtP2Block) void k_ht_p2(HtPass2Args a) {
    __builtin_amdgcn_s_setprio(3);   // R's chain: issue ahead of the persistent S pass 1 sharing the SIMD
    constexpr uint32_t B = kHtP2Block, U = kHtP2Items;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);                 // [nb2] counts
    uint32_t* cur = cnt + a.nb2;                                        // [nb2] cursors
    uint64_t* sorted = reinterpret_cast<uint64_t*>(cur + a.nb2);        // [kHtP2Keep] d2 order (KEEP)
    __shared__ uint32_t tmp[B / 64];
    const uint32_t d1 = blockIdx.x, tid = threadIdx.x, nb2 = a.nb2;
    const uint32_t lo = a.hist1[static_cast<size_t>(d1) * a.nt1];
    const uint32_t hi = d1 + 1 < a.nb1 ? a.hist1[static_cast<size_t>(d1 + 1) * a.nt1] : a.n, m = hi - lo;
    const bool keep = KEEP && m <= kHtP2Keep;   // workgroup-uniform
    auto d2_of = [&](uint64_t c) { return static_cast<uint32_t>(q_from_hash(c, a.f2)) & a.f2.dmask; };
    for (uint32_t d = tid; d < nb2; d += B) cnt[d] = 0;
    __syncthreads();
    uint64_t c[U];
    for (uint32_t f0 = lo; f0 < hi; f0 += B * U) {
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t f = f0 + u * B + tid;
            c[u] = f < hi ? static_cast<uint64_t>(a.codes[f]) : 0;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) count_digit(cnt, d2_of(c[u]), f0 + u * B + tid < hi);
    }
    __syncthreads();
    {   // exclusive scan of the counts: nb2 / B consecutive digits per thread
        const uint32_t per = (nb2 + B - 1) / B, d0 = tid * per;
        uint32_t local = 0;
        for (uint32_t j = 0; j < per; j++)
            if (d0 + j < nb2) local += cnt[d0 + j];
        uint32_t tot;
        uint32_t run = block_exclusive_scan_t<B / 64>(local, tmp, tot);
        for (uint32_t j = 0; j < per; j++) {
            const uint32_t d = d0 + j;
            if (d < nb2) {
                a.bounds[static_cast<size_t>(d1) * nb2 + d] = lo + run;
                cur[d] = keep ? run : lo + run;
                run += cnt[d];
            }
        }
        if (d1 + 1 == a.nb1 && tid == 0) a.bounds[static_cast<size_t>(a.nb1) * nb2] = hi;
    }
    __syncthreads();
    if (keep) {   // the run is in c[] (one round of the loop above)
#pragma unroll
        for (uint32_t u = 0; u < U; u++)
            if (u * B + tid < m) sorted[atomicAdd(&cur[d2_of(c[u])], 1u)] = c[u];
        __syncthreads();
        for (uint32_t i = tid; i < m; i += B) a.out[lo + i] = static_cast<int64_t>(sorted[i]);
        return;
    }
    for (uint32_t f0 = lo; f0 < hi; f0 += B * U) {
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t f = f0 + u * B + tid;
            c[u] = f < hi ? static_cast<uint64_t>(a.codes[f]) : 0;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t f = f0 + u * B + tid;
            const uint32_t r = agg_rank(cur, d2_of(c[u]), f < hi);
            if (f < hi) a.out[r] = static_cast<int64_t>(c[u]);
        }
    }
}

// The tables over `nseg` build segments (codes in partition order + bounds).
struct HtArgs {
    const int64_t* codes[kHtSegs];
    const uint32_t* bounds[kHtSegs];   // P + 1 each
    uint32_t nseg, nb1, nb2, pad;
    uint64_t e1;                       // E_0 (ht_empty)
    uint64_t* table;                   // slots (4 |R| + 2 P bound)
    uint2* desc;                       // per final partition: {slot base (even), buckets - 1}, written by k_ht_fill
    const uint32_t* uni;               // nullptr, or {1, cap}: every partition gets cap slots at p * cap (k_np_ct_plan)
};

__device__ __forceinline__ uint32_t ht_part_size(const HtArgs& a, uint32_t p) {
    uint32_t lo[kHtSegs], hi[kHtSegs];   // every segment's bounds requested together
#pragma unroll
    for (uint32_t g = 0; g < kHtSegs; g++) {
        lo[g] = g < a.nseg ? a.bounds[g][p] : 0u;
        hi[g] = g < a.nseg ? a.bounds[g][p + 1] : 0u;
    }
    uint32_t m = 0;
#pragma unroll
    for (uint32_t g = 0; g < kHtSegs; g++) m += hi[g] - lo[g];
    return m;
}

__device__ __forceinline__ void ht_insert(uint64_t* tab, uint32_t bmask, uint64_t e, uint64_t c) {
    uint32_t b = static_cast<uint32_t>(c >> kHtBucketShift) & bmask;
    for (;;) {
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const uint64_t old = atomicCAS(reinterpret_cast<unsigned long long*>(tab + 2 * b + j), e, c);
            if (old == e || old == c) return;   // placed, or already there (duplicates stored once)
        }
        b = (b + 1) & bmask;
    }
}

// A workgroup per kHtPpw consecutive partitions (their bounds in every
// segment staged in LDS in one round of loads), each wave builds partitions
// w, w + 4, ... in its LDS table slice: the partition's codes (<= 8 per lane,
// flattened over the segments) are all requested at once, every code claims a
// slot of its home bucket with a 32-bit counter (slot 0 before slot 1, as the
// probe assumes), codes finding their home bucket full (~7 % at load 2/3)
// probe onwards with compare-and-swap, and the table is written out in 16-B
// stores. Duplicates may take two slots: harmless to a set test, and the cap
// counts them.
template <bool ONE>   // ONE: a single build segment (one device): element r is at codes[0] + start + r
__global__ __launch_bounds__(256) void k_ht_fill(HtArgs a) {
    __builtin_amdgcn_s_setprio(3);   // R's chain: issue ahead of the persistent S pass 1 sharing the SIMD
    // codes per lane: a partition that fits the slice at load <= 0.8 (the
    // uniform layout's bound; the radix layout's caps keep it <= 2/3)
    constexpr uint32_t CPL = kHtLcap * 4 / 5 / 64 + 1;
    __shared__ __attribute__((aligned(16))) uint64_t wtab[4][kHtLcap];
    __shared__ uint32_t wcnt[4][kHtLcap / 2];      // per-wave bucket fill counters
    __shared__ uint32_t sb[kHtSegs][kHtPpw + 1];   // bounds of the workgroup's partitions, per segment
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t nseg = a.nseg;
    const uint32_t P = a.nb1 * a.nb2;
    const uint32_t p0 = blockIdx.x * kHtPpw, np = min(P - p0, kHtPpw);
    for (uint32_t t = tid; t < nseg * (kHtPpw + 1); t += 256) {
        const uint32_t g = t / (kHtPpw + 1), j = t - g * (kHtPpw + 1);
        sb[g][j] = a.bounds[g][p0 + min(j, np)];
    }
    __syncthreads();
    for (uint32_t j = wave; j < np; j += 4) {
        const uint32_t p = p0 + j;
        const uint64_t e = ht_empty(p, a.e1);
        // lane g < nseg: segment g's run of p; x = inclusive prefix of the run
        // lengths, base = where element r of p sits in segment g, minus r
        const uint32_t len = lane < nseg ? sb[lane][j + 1] - sb[lane][j] : 0u;
        uint32_t x = len;
#pragma unroll
        for (int o = 1; o < kHtSegs; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= static_cast<uint32_t>(o)) x += y;
        }
        const uint64_t base = lane < nseg ? reinterpret_cast<uint64_t>(a.codes[lane] + sb[lane][j]) - 8ull * (x - len) : 0ull;
        uint32_t b0 = lane < nseg ? sb[lane][j] : 0u;
#pragma unroll
        for (int o = 1; o < kHtSegs; o <<= 1) b0 += __shfl_xor(b0, o, 64);
        const uint32_t bstart = __builtin_amdgcn_readfirstlane(b0);   // the partition's first code over all segments
        const uint32_t m = __builtin_amdgcn_readlane(x, nseg - 1);
        const uint32_t base_lo = static_cast<uint32_t>(base), base_hi = static_cast<uint32_t>(base >> 32);
        // the table's slots: closed form from the partition's start (a cap is
        // at most 4 m + 2 slots), or p * cap in the uniform layout
        uint2 ds;
        if (a.uni && a.uni[0]) ds = make_uint2(p * a.uni[1], a.uni[1] / 2 - 1u);
        else ds = make_uint2(4 * bstart + 2 * p, ht_cap(m) / 2 - 1u);
        if (lane == 0) a.desc[p] = ds;
        const uint32_t cap = 2 * (ds.y + 1);
        uint64_t* out = a.table + ds.x;
        // element r lies in the last segment g whose run starts at or before r:
        // a binary search over the run ends held lane-wise (lane k: x_k). The
        // cross-lane reads need every lane active: src_of is only called
        // outside divergent branches (r clamped, the load conditional after)
        auto src_of = [&](uint32_t r) -> const int64_t* {
            if constexpr (ONE) return a.codes[0] + sb[0][j] + r;
            int g = 0;
#pragma unroll
            for (int step = kHtSegs / 2; step >= 1; step >>= 1) {
                const int cand = g + step;
                const uint32_t xv = __shfl(x, cand - 1, 64);
                if (static_cast<uint32_t>(cand) < nseg && xv <= r) g = cand;
            }
            const uint32_t lo32 = __shfl(base_lo, g, 64), hi32 = __shfl(base_hi, g, 64);
            return reinterpret_cast<const int64_t*>((static_cast<uint64_t>(hi32) << 32) | lo32) + r;
        };
        if (cap <= kHtLcap && m <= CPL * 64) {
            uint64_t c[CPL];
#pragma unroll
            for (uint32_t i = 0; i < CPL; i++) {
                const uint32_t r = i * 64 + lane;
                const int64_t* src = src_of(min(r, m - 1u));   // every lane (m >= 1 when any loads)
                c[i] = r < m ? static_cast<uint64_t>(*src) : 0ull;
            }
            uint32_t* bc = wcnt[wave];
            for (uint32_t sl = lane; sl < cap; sl += 64) wtab[wave][sl] = e;
            for (uint32_t b = lane; b < cap / 2; b += 64) bc[b] = 0;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_wave_barrier();
            uint32_t ovf = 0;   // bit i: c[i] found its home bucket full
#pragma unroll
            for (uint32_t i = 0; i < CPL; i++) {
                if (i * 64 + lane < m) {
                    const uint32_t b = static_cast<uint32_t>(c[i] >> kHtBucketShift) & ds.y;
                    const uint32_t k = atomicAdd(&bc[b], 1u);
                    if (k < 2) wtab[wave][2 * b + k] = c[i];
                    else ovf |= 1u << i;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (uint32_t i = 0; i < CPL; i++) {
                if ((ovf >> i) & 1u) {
                    uint32_t b = static_cast<uint32_t>(c[i] >> kHtBucketShift) & ds.y;
                    for (bool placed = false; !placed;) {
                        b = (b + 1) & ds.y;
#pragma unroll
                        for (int k = 0; k < 2 && !placed; k++) {
                            const uint64_t old = atomicCAS(reinterpret_cast<unsigned long long*>(&wtab[wave][2 * b + k]), e, c[i]);
                            placed = old == e || old == c[i];
                        }
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_wave_barrier();
            ulonglong2* o2 = reinterpret_cast<ulonglong2*>(out);
            const ulonglong2* t2 = reinterpret_cast<const ulonglong2*>(wtab[wave]);
            for (uint32_t b = lane; b < cap / 2; b += 64) o2[b] = t2[b];
        } else {   // a partition beyond the slice (adversarial inputs): device atomics in place
            for (uint32_t sl = lane; sl < cap; sl += 64) out[sl] = e;
            __threadfence();
            __builtin_amdgcn_wave_barrier();
            for (uint32_t r0 = 0; r0 < m; r0 += 64) {   // wave-uniform trip count
                const uint32_t r = r0 + lane;
                const int64_t* src = src_of(min(r, m - 1u));
                if (r < m) ht_insert(out, ds.y, e, static_cast<uint64_t>(*src));
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------
// On-chip probe: the probe side's pass 2 never lands in HBM. Persistent: XCD x
// walks tiles [x, x + 1) * ntiles / 8 of the pass-1 output (tiles of one d1 are
// contiguous, so an XCD's L2 holds the few d1 regions it probes), its
// workgroups round-robin over them. Per 4096-key tile, three barriers:
//   rank by d2 (agg_rank: LDS atomics, aggregated over a wave's lanes that
//   share a digit, so a hot key does not serialise) | B1 | one wave scans the
//   counts | B2 | scatter into skey (grouped by d2: neighbouring lanes probe
//   the same small table, mostly the same cache line), issue the next tile's
//   loads, clear the other counter row, stage the other descriptor buffer for
//   the next tile's d1 | B3 | probe: every lane requests all its items' home
//   buckets at once (only the 16-B buckets stay in registers; codes and
//   descriptors are re-read from LDS), then items whose home bucket is full
//   without a match walk on.
// Counters and descriptors are double-buffered, so the next tile's ranking may
// start while slower waves still probe this one (its scatter waits behind the
// next B1 / B2, which every wave reaches only after its probe).
// HK = kHashed when the pass-1 output holds codes (k_chunk_codes), else the key is
// hashed here (a stable pass 1 of whole tuples).
// ---------------------------------------------------------------------------
struct HtProbeArgs {
    PassArgs a;                  // the pass-2 tile mapping over the pass-1 output
    const uint2* desc;
    const uint64_t* table;
    unsigned long long* count;   // {count, failed}: failed = 1 when the pass-1 error word is set
    const uint32_t* err;         // S's pass-1 error word (chunk_err_word), or null
    uint64_t seed;
    uint64_t e1;                 // E_0 (ht_empty)
    uint32_t nb2;
    uint32_t pad;
};

// The chunked pass 1's error word folded into the count pair by the probe
// (read after k_tile_chunks, which also reports into it).
__device__ __forceinline__ void fold_pass1_error(const uint32_t* err, unsigned long long* count) {
    if (err && blockIdx.x == 0 && threadIdx.x == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicOr(count + 1, 1ull);
}

constexpr int kProbeBlock = 1024, kProbeItems = 4;   // 16 waves, 4 keys per lane: a 4096-key tile

__host__ __device__ constexpr size_t probe_ht_lds_bytes(int T, uint32_t nb) {
    return static_cast<size_t>(T + 2) * 8 + static_cast<size_t>(nb) * 2 * 12 + 64;
}

// Exclusive scan of nb digit counts C[0, nb) in place by one wave; returns the
// total on every lane.
__device__ __forceinline__ uint32_t wave_scan_counts(uint32_t* C, uint32_t nb, uint32_t lane) {
    if (nb == 256) {   // the common 8-bit d2: one 16-B LDS read per lane
        const uint4 q = reinterpret_cast<uint4*>(C)[lane];
        const uint32_t local = q.x + q.y + q.z + q.w;
        uint32_t x = local;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= static_cast<uint32_t>(o)) x += y;
        }
        const uint32_t r0 = x - local;
        reinterpret_cast<uint4*>(C)[lane] = make_uint4(r0, r0 + q.x, r0 + q.x + q.y, r0 + q.x + q.y + q.z);
        return __shfl(x, 63, 64);
    }
    const uint32_t per = (nb + 63) / 64, d0 = lane * per;
    uint32_t local = 0;
    for (uint32_t j = 0; j < per; j++)
        if (d0 + j < nb) local += C[d0 + j];
    uint32_t x = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= static_cast<uint32_t>(o)) x += y;
    }
    uint32_t run = x - local;
    for (uint32_t j = 0; j < per; j++)
        if (d0 + j < nb) {
            const uint32_t c = C[d0 + j];
            C[d0 + j] = run;
            run += c;
        }
    return __shfl(x, 63, 64);
}

// FORM bit 0 (kProbeRadix): the radix digit of a code is a plain bit field,
// d2 = (c >> shift) & dmask (no h % P, no sub-partition bits); bit 1
// (kProbeChunked): the input is the chunked keys-only pass 1 (a code column,
// tile t = chunk [tile_start[t], + tile_cnt[t])). Both drop the run-time mode
// branches and the kernel-argument state they keep live.
constexpr int kProbeRadix = 1, kProbeChunked = 2;

template <int BLOCK, int ITEMS, int HK, int FORM = 0>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8))) void k_probe_ht(HtProbeArgs pa) {
    constexpr int T = BLOCK * ITEMS;
    constexpr bool RADIX = (FORM & kProbeRadix) != 0, CHUNKED = (FORM & kProbeChunked) != 0;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const PassArgs& a = pa.a;
    const uint32_t nb = a.nbins;
    int64_t* skey = reinterpret_cast<int64_t*>(smem);              // [T + 2]: slot T takes invalid lanes' writes
    uint2* sdesc = reinterpret_cast<uint2*>(skey + T + 2);         // [2][nb]
    uint32_t* cntb = reinterpret_cast<uint32_t*>(sdesc + 2 * nb);   // [2][nb]
    __shared__ uint32_t red[BLOCK / 64];
    __shared__ uint32_t tot_s;

    const uint32_t total = a.tile_base[a.nseg];
    const uint32_t xcd = blockIdx.x & 7u, g8 = gridDim.x >> 3;
    const uint32_t t_lo = static_cast<uint32_t>(static_cast<uint64_t>(total) * xcd / 8);
    const uint32_t t_hi = static_cast<uint32_t>(static_cast<uint64_t>(total) * (xcd + 1) / 8);
    uint32_t tile = t_lo + (blockIdx.x >> 3);
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    uint32_t hits = 0;
    if (tile < t_hi) {   // block-uniform
        const uint32_t wbase = wave * 64 * ITEMS;
        const longlong2* rel = reinterpret_cast<const longlong2*>(a.in_keys);
        const bool soa = CHUNKED || a.in_pays != nullptr || a.keys_only;
        auto d2_of = [&](uint64_t c) -> uint32_t {
            if constexpr (RADIX) return static_cast<uint32_t>(c >> a.f.shift) & a.f.dmask;
            return static_cast<uint32_t>(q_from_hash(c, a.f) >> a.f.shift) & a.f.dmask;
        };
        int64_t key[ITEMS];
        uint32_t vm = 0, d1 = 0;
        auto load = [&](uint32_t t, uint32_t& m, uint32_t& d) {
            d = a.tile_seg[t];
            m = 0;
            uint32_t lo, c;
            if constexpr (CHUNKED) {
                lo = a.tile_start[t];
                c = a.tile_cnt[t];
            } else {
                TileLoc L;
                locate_tile<T>(a, t, L);
                lo = L.lo;
                c = L.hi - L.lo;
            }
            // unconditional loads (clamped: a tile holds >= 1 code), no select
            // on a loaded value
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                const uint32_t e = wbase + i * 64 + lane;
                const uint32_t ix = lo + min(e, c - 1u);
                // nontemporal: the code stream (read once) does not displace
                // the d1 tables the XCD's L2 holds for the probes
                key[i] = soa ? __builtin_nontemporal_load(a.in_keys + ix) : __builtin_nontemporal_load(&rel[ix].x);
                m |= e < c ? (1u << i) : 0u;
            }
        };
        auto stage = [&](uint32_t buf, uint32_t dd) {
            for (uint32_t d = tid; d < nb; d += BLOCK) sdesc[buf * nb + d] = pa.desc[static_cast<size_t>(dd) * pa.nb2 + d];
        };
        load(tile, vm, d1);
        uint32_t sd[2] = {d1, 0xffffffffu};   // d1 staged in each descriptor buffer
        stage(0, d1);
        for (uint32_t d = tid; d < nb; d += BLOCK) cntb[d] = 0;
        __syncthreads();
        uint32_t buf = 0;
        for (;;) {
            uint32_t* C = cntb + buf * nb;
            const uint2* D = sdesc + buf * nb;
            uint32_t dig[ITEMS], rank[ITEMS];
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                const uint64_t h = hash64<HK>(static_cast<uint64_t>(key[i]), pa.seed);
                key[i] = static_cast<int64_t>(h);
                dig[i] = d2_of(h);
                rank[i] = agg_rank(C, dig[i], (vm >> i) & 1u);
            }
            __syncthreads();   // B1
            if (wave == 0) {   // exclusive scan of the counts by one wave
                const uint32_t t = wave_scan_counts(C, nb, lane);
                if (lane == 0) tot_s = t;
            }
            __syncthreads();   // B2
            const uint32_t cnt = tot_s;
            uint32_t pos[ITEMS];
#pragma unroll
            for (int i = 0; i < ITEMS; i++) pos[i] = C[dig[i]] + rank[i];

            // branch-free: slot T takes invalid lanes' writes (a sink)
#pragma unroll
            for (int i = 0; i < ITEMS; i++) skey[((vm >> i) & 1u) ? pos[i] : static_cast<uint32_t>(T)] = key[i];
            const uint32_t next = tile + g8;
            const bool more = next < t_hi;
            uint32_t nvm = 0, nd1 = d1;
            // the next tile's codes, counter row and descriptors
            if (more) load(next, nvm, nd1);
            const uint32_t ob = buf ^ 1u;
            for (uint32_t d = tid; d < nb; d += BLOCK) cntb[ob * nb + d] = 0;
            if (more && sd[ob] != nd1) {
                stage(ob, nd1);
                sd[ob] = nd1;
            }
            __syncthreads();   // B3
            // probe: all items' home buckets in flight at once, then the walks
            const uint64_t e0 = d1 == 0 ? pa.e1 : 0ull;   // E of partition (d1, d2): e1 only for partition 0
            const ulonglong2* tab2 = reinterpret_cast<const ulonglong2*>(pa.table);
            ulonglong2 v[ITEMS];
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {   // unconditional: an unused lane reads code 0's bucket
                const uint32_t k = i * BLOCK + tid;
                const uint64_t c = k < cnt ? static_cast<uint64_t>(skey[k]) : 0ull;
                const uint2 ds = D[d2_of(c)];
                v[i] = tab2[(ds.x >> 1) + (static_cast<uint32_t>(c >> kHtBucketShift) & ds.y)];
            }
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                const uint32_t k = i * BLOCK + tid;
                if (k < cnt) {
                    const uint64_t c = static_cast<uint64_t>(skey[k]);
                    bool hit = v[i].x == c || v[i].y == c;
                    const uint32_t d2 = d2_of(c);
                    const uint64_t e = d2 == 0 ? e0 : 0ull;
                    if (!hit && v[i].y != e) {   // home bucket full, no match: walk on
                        const uint2 ds = D[d2];
                        uint32_t b = static_cast<uint32_t>(c >> kHtBucketShift) & ds.y;
                        for (;;) {
                            b = (b + 1) & ds.y;
                            const ulonglong2 w = tab2[(ds.x >> 1) + b];
                            hit = w.x == c || w.y == c;
                            if (hit || w.y == e) break;
                        }
                    }
                    hits += hit ? 1u : 0u;
                }
            }
            if (!more) break;
            tile = next;
            vm = nvm;
            d1 = nd1;
            buf = ob;
        }
    }
    uint32_t x = hits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if (lane == 0) red[wave] = x;
    __syncthreads();
    if (tid == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < BLOCK / 64; w++) t += red[w];
        if (t) atomicAdd(pa.count, t);
    }
    fold_pass1_error(pa.err, pa.count);
}

// ---------------------------------------------------------------------------
// NoPartitioning over code tables (the count probe of join_nopart, PHJ_NP_CT):
// the reference's one global table (src/NoPartitioning/HashJoin.hpp:76-126)
// is realised as 2^k small code tables, region p = the low k bits of the code
// (the layout k_np_build_region already used), built by R's two-pass code
// partition and k_ht_fill. S is NOT partitioned: every S key hashes, picks its
// region's table and reads one 16-B bucket, as the reference's Probe()
// (:128-187) reads its table. With every region at most 0.8 full at a common
// power-of-two cap (k_np_ct_plan decides on the device), region p sits at
// slot p * cap and the probe computes its bucket with no descriptor read;
// otherwise (skewed build keys) it reads desc[p] like k_probe_ht.
// ---------------------------------------------------------------------------

// One workgroup: the largest region, then {uniform?, cap}.
__global__ __launch_bounds__(256) void k_np_ct_plan(const uint32_t* bounds, uint32_t P, uint64_t slot_bound,
                                                    uint32_t* uni) {
    __shared__ uint32_t red[4];
    uint32_t mx = 0;
    for (uint32_t p = threadIdx.x; p < P; p += 256) mx = max(mx, bounds[p + 1] - bounds[p]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, static_cast<uint32_t>(__shfl_xor(mx, o, 64)));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        mx = max(max(red[0], red[1]), max(red[2], red[3]));
        uint32_t cap = 2;
        while (cap < mx + (mx + 3) / 4) cap <<= 1;   // load <= 0.8 in every region
        const bool ok = static_cast<uint64_t>(cap) * P <= slot_bound && cap <= kHtLcap;
        uni[0] = ok ? 1u : 0u;
        uni[1] = cap;
    }
}

template <int HK, int ITEMS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_np_probe_ct(
    const longlong2* S, uint64_t nS, const uint64_t* table, const uint2* desc, const uint32_t* uni, uint32_t P,
    uint64_t seed, uint64_t e1, unsigned long long* count) {
    const bool uniform = __builtin_amdgcn_readfirstlane(uni[0]) != 0;
    const uint32_t nbk = __builtin_amdgcn_readfirstlane(uni[1]) / 2;   // buckets per region (uniform)
    const ulonglong2* tab2 = reinterpret_cast<const ulonglong2*>(table);
    const uint32_t tid = threadIdx.x;
    uint32_t hits = 0;
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * 256 * ITEMS;
    // the probe loop is instantiated per layout: a descriptor load that the
    // uniform layout does not need, speculated by the compiler, put a wait for
    // every earlier load in front of each item's bucket read (the items' reads
    // then went out one at a time)
    auto run = [&](auto UNI) {
        constexpr bool UNIFORM = decltype(UNI)::value;
        for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * 256 * ITEMS; base < nS; base += step) {
            uint64_t c[ITEMS];
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {   // S streams past the caches' allocate (it is read once)
                const uint64_t ix = min(base + i * 256 + tid, nS - 1);
                c[i] = static_cast<uint64_t>(__builtin_nontemporal_load(&S[ix].x));
            }
            uint32_t bb[ITEMS], bm[ITEMS], bk[ITEMS];
            ulonglong2 v[ITEMS];
            if constexpr (!UNIFORM) {   // every descriptor requested before any bucket
                uint2 ds[ITEMS];
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    c[i] = hash64<HK>(c[i], seed);
                    ds[i] = desc[static_cast<uint32_t>(c[i]) & (P - 1)];
                }
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    bb[i] = ds[i].x >> 1;
                    bm[i] = ds[i].y;
                }
            } else {
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    c[i] = hash64<HK>(c[i], seed);
                    bb[i] = (static_cast<uint32_t>(c[i]) & (P - 1)) * nbk;
                    bm[i] = nbk - 1;
                }
            }
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                bk[i] = static_cast<uint32_t>(c[i] >> kHtBucketShift) & bm[i];
                v[i] = tab2[bb[i] + bk[i]];
            }
            // branch-free (a short-circuit || let the compiler split the last
            // item's 16-B read into two dependent 8-B reads)
            uint32_t pend = 0;   // bit i: item i's home bucket is full without a match
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                const uint32_t valid = base + i * 256 + tid < nS ? 1u : 0u;
                const uint64_t e = ht_empty(static_cast<uint32_t>(c[i]) & (P - 1), e1);
                const uint32_t hit = static_cast<uint32_t>(v[i].x == c[i]) | static_cast<uint32_t>(v[i].y == c[i]);
                hits += hit & valid;
                pend |= (valid & (hit ^ 1u) & static_cast<uint32_t>(v[i].y != e)) << i;
            }
            // the walks: every pending item's next bucket in flight at once (loads
            // unconditional: a settled item re-reads its last bucket)
            while (pend) {
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    if ((pend >> i) & 1u) bk[i] = (bk[i] + 1) & bm[i];
                    v[i] = tab2[bb[i] + bk[i]];
                }
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    const uint32_t pi = (pend >> i) & 1u;
                    const uint64_t e = ht_empty(static_cast<uint32_t>(c[i]) & (P - 1), e1);
                    const uint32_t hit = static_cast<uint32_t>(v[i].x == c[i]) | static_cast<uint32_t>(v[i].y == c[i]);
                    const uint32_t done = pi & (hit | static_cast<uint32_t>(v[i].y == e));
                    hits += done & hit;
                    pend &= ~(done << i);
                }
            }
        }
    };
    if (uniform) run(std::true_type{});
    else run(std::false_type{});
    __shared__ uint32_t red[4];
    uint32_t x = hits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = x;
    __syncthreads();
    if (tid == 0) {
        const unsigned long long t = static_cast<unsigned long long>(red[0]) + red[1] + red[2] + red[3];
        if (t) atomicAdd(count, t);
    }
}

// ---------------------------------------------------------------------------
// Test hook (phj_probe_pass1): the pass-1 tiles the probe consumes,
// concatenated in tile order. cnt[t] = keys of tile t (0 past the last tile);
// after an exclusive scan, k_gather_pass1 copies tile t to out[off[t], ...).
// ---------------------------------------------------------------------------
template <int T>
__global__ __launch_bounds__(256) void k_tile_counts(PassArgs a, uint32_t nt, uint32_t* cnt) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t > nt) return;
    TileLoc L;
    cnt[t] = (t < nt && locate_tile<T>(a, t, L)) ? L.hi - L.lo : 0u;
}

template <int T>
__global__ __launch_bounds__(256) void k_gather_pass1(PassArgs a, const uint32_t* off, int64_t* out) {
    TileLoc L;
    if (!locate_tile<T>(a, blockIdx.x, L)) return;
    const bool soa = a.in_pays != nullptr || a.keys_only;
    const longlong2* rel = reinterpret_cast<const longlong2*>(a.in_keys);
    int64_t* o = out + off[blockIdx.x];
    for (uint32_t e = threadIdx.x; e < L.hi - L.lo; e += 256) o[e] = soa ? a.in_keys[L.lo + e] : rel[L.lo + e].x;
}

}  // namespace phj
