// phj_join.h — build / probe / count kernels for gfx950.
//
// Radix path (src/RadixCluster/HashJoin.hpp:243-331, Join()):
//   k_join_prep + batched scan : per-partition table sizes and probe work items
//   k_build                    : one workgroup per partition builds a
//                                bucket-chained table in compacted (CSR) form:
//                                bucket b of partition p holds the keys
//                                tkeys[tkb[p] + toffs[tob[p]+b] .. +toffs[..+b+1]).
//                                LDS counting sort for small partitions, global
//                                atomics for partitions past the LDS capacity.
//   k_probe                    : persistent workgroups walk (partition, S-chunk)
//                                items; a partition's table is staged into LDS
//                                once per item, every S key probes it and the
//                                first equal key counts (Get() returns the first
//                                match, LinearProbing.hpp:160-180).
// Skew is handled by the item split: a hot partition becomes many S chunks.
//
// NoPartitioning path (src/NoPartitioning/HashJoin.hpp:76-187):
//   k_np_build_region / k_np_probe : one global bucketized linear-probing table in
//                                HBM, 64-B buckets {7 keys, fill count}. As in
//                                LinearProbing.hpp:22-83 occupancy is a
//                                per-bucket fill counter (no sentinel key: every
//                                int64 is a valid key), inserts claim a slot
//                                with an atomic on the counter and move to the
//                                next bucket when full, and a lookup stops at
//                                the first non-full bucket.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "phj_hash.h"
#include "phj_pow.h"
#include "phj_partition.h"

namespace phj {

constexpr int kMaxSegs = 16;
constexpr int kBuildKPL = 8;   // k_build_small: R tuples per lane (64 * 8 = 512 per partition)
constexpr int kProbeWaveKPL = 8;     // k_probe_wave: S keys per lane per item (512 per item)
constexpr int kProbeWaveTcap = 512;  // k_probe_wave: staged table keys per wave

struct Seg {
    const int64_t* keys;
    const int64_t* pays;
    const uint32_t* bounds;
};

struct SegList {
    Seg seg[kMaxSegs];
    uint32_t nseg;
    uint32_t P;
};

__host__ __device__ __forceinline__ uint32_t table_buckets(uint32_t m) {
    if (m <= 1) return 1u;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t np2 = 1u << (32 - __clz(m - 1));
#else
    uint32_t np2 = 1;
    while (np2 < m) np2 <<= 1;
#endif
    return np2 >> 1;
}

__device__ __forceinline__ uint32_t bucket_of(uint64_t h, uint32_t nbk) {
    return static_cast<uint32_t>(h >> 32) & (nbk - 1u);
}

// arr: 3 arrays of P+1 entries: m_p, NB_p + 1, items_p (last entry 0).
__global__ __launch_bounds__(kBlock) void k_join_prep(SegList L, const uint32_t* sbounds,
                                                      uint32_t chunk, uint32_t* arr) {
    const uint32_t P = L.P;
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (p > P) return;
    const size_t stride = static_cast<size_t>(P) + 1;
    if (p == P) {
        arr[P] = 0;
        arr[stride + P] = 0;
        arr[2 * stride + P] = 0;
        return;
    }
    uint32_t m = 0;
    for (uint32_t g = 0; g < L.nseg; g++) m += L.seg[g].bounds[p + 1] - L.seg[g].bounds[p];
    const uint32_t s = sbounds[p + 1] - sbounds[p];
    arr[p] = m;
    arr[stride + p] = table_buckets(m) + 1;
    arr[2 * stride + p] = (m && s) ? (s + chunk - 1) / chunk : 0u;
}

// A probe work item: one S chunk of one partition plus where that partition's
// table lives, so a probing workgroup needs a single 32-B descriptor load.
struct ProbeItem {
    uint32_t s_lo, s_cnt;   // S keys [s_lo, s_lo + s_cnt)
    uint32_t kb, m;         // table keys [kb, kb + m)
    uint32_t ob, nbk;       // bucket offsets [ob, ob + nbk]
    uint32_t pad0, pad1;
};

// One wave per partition writes its (partition, chunk) work items.
__global__ __launch_bounds__(kBlock) void k_items_expand(const uint32_t* itb, const uint32_t* tkb,
                                                         const uint32_t* tob, const uint32_t* sbounds,
                                                         uint32_t P, uint32_t chunk, ProbeItem* items) {
    const uint32_t p = blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (p >= P) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lo = itb[p], hi = itb[p + 1];
    if (lo == hi) return;
    const uint32_t kb = tkb[p], m = tkb[p + 1] - kb;
    const uint32_t ob = tob[p], nbk = tob[p + 1] - ob - 1;
    const uint32_t sb = sbounds[p], se = sbounds[p + 1];
    for (uint32_t i = lo + lane; i < hi; i += 64) {
        ProbeItem it;
        it.s_lo = sb + (i - lo) * chunk;
        it.s_cnt = min(chunk, se - it.s_lo);
        it.kb = kb;
        it.m = m;
        it.ob = ob;
        it.nbk = nbk;
        it.pad0 = it.pad1 = 0;
        items[i] = it;
    }
}

struct BuildArgs {
    SegList L;
    const uint32_t* tkb;   // P+1: table key base (exclusive scan of m_p)
    const uint32_t* tob;   // P+1: table offset base (exclusive scan of NB_p + 1)
    int64_t* tkeys;
    int64_t* tpays;
    uint32_t* toffs;
    uint32_t* gcursor;     // global cursors for partitions beyond the LDS capacity
    uint32_t* biglist;     // partitions left to k_build_big
    uint32_t* bigcount;    // (zeroed before k_build_small)
    uint32_t ocap;         // LDS bucket-counter capacity (per wave in k_build_small)
    uint32_t pad;
    uint64_t seed;
};

// LDS ordering between lanes of one wave (stores before loads of other lanes).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// One wave per partition: bucket counting sort of R_p in the wave's LDS slice
// (the common case: R_p ~ |R| / P tuples). R_p may arrive as up to 16 build
// segments (the shards of every rank after the multi-GPU all-gather): lane g
// loads segment g's bounds, a wave prefix over the segment sizes maps every
// flat index of R_p to (segment, row), and all of R_p is loaded ONCE into
// registers (KPL tuples per lane) and hashed once; counting, the bucket scan
// and the placement then run from registers and LDS. Partitions with more than
// 64 * KPL tuples or a bucket array beyond the wave's LDS slice are appended to
// biglist for k_build_big. The order inside a bucket is irrelevant to the
// semi-join count (set membership).
template <int HK, int KPL>
__global__ __launch_bounds__(kBlock) void k_build_small(BuildArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(smem) + wave * a.ocap;
    const uint32_t P = a.L.P, nseg = a.L.nseg;
    const uint32_t nw = gridDim.x * kWaves;
    // lane g < nseg holds segment g's columns
    const int64_t* skeys = lane < nseg ? a.L.seg[lane].keys : nullptr;
    const int64_t* spays = lane < nseg ? a.L.seg[lane].pays : nullptr;
    // key-only build segments (the multi-GPU exchange ships keys): no payloads
    // to copy; every probe only tests key equality
    const bool spays_all = a.L.seg[0].pays != nullptr;
    const uint32_t* sbnd = lane < nseg ? a.L.seg[lane].bounds : nullptr;
    for (uint32_t p = blockIdx.x * kWaves + wave; p < P; p += nw) {
        // table bases and the segments' bounds in one round of loads
        uint32_t lo = 0, c = 0;
        if (lane < nseg) {
            lo = sbnd[p];
            c = sbnd[p + 1] - lo;
        }
        const uint32_t kb = a.tkb[p], m = a.tkb[p + 1] - kb;
        const uint32_t ob = a.tob[p], nbk = a.tob[p + 1] - ob - 1;
        uint32_t* offs = a.toffs + ob;
        if (m == 0) {
            for (uint32_t i = lane; i <= nbk; i += 64) offs[i] = 0;
            continue;
        }
        if (nbk > a.ocap || m > 64u * KPL) {
            if (lane == 0) a.biglist[atomicAdd(a.bigcount, 1u)] = p;
            continue;
        }
        uint32_t inc = c;   // inclusive prefix of the segment sizes (lanes < 16)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= static_cast<uint32_t>(o)) inc += y;
        }
        const int64_t rowoff = static_cast<int64_t>(lo) - static_cast<int64_t>(inc - c);   // row = flat + rowoff
        int64_t key[KPL], pay[KPL];
        uint32_t bkt[KPL];
#pragma unroll
        for (int j = 0; j < KPL; j++) {
            const uint32_t f = j * 64 + lane;
            uint32_t g = 0;
            for (uint32_t l = 0; l + 1 < nseg; l++) g += f >= static_cast<uint32_t>(__shfl(inc, l, 64)) ? 1u : 0u;
            const int64_t ro = __shfl(rowoff, static_cast<int>(g), 64);
            const int64_t* kp = reinterpret_cast<const int64_t*>(__shfl(reinterpret_cast<intptr_t>(skeys), static_cast<int>(g), 64));
            const int64_t* pp = reinterpret_cast<const int64_t*>(__shfl(reinterpret_cast<intptr_t>(spays), static_cast<int>(g), 64));
            key[j] = 0;
            pay[j] = 0;
            if (f < m) {
                const int64_t row = static_cast<int64_t>(f) + ro;
                key[j] = kp[row];
                if (pp) pay[j] = pp[row];
            }
        }
        for (uint32_t i = lane; i < nbk; i += 64) cnt[i] = 0;
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < KPL; j++) {
            const uint64_t h = hash64<HK>(static_cast<uint64_t>(key[j]), a.seed);
            bkt[j] = bucket_of(h, nbk);
            if (j * 64 + lane < m) atomicAdd(&cnt[bkt[j]], 1u);
        }
        wave_lds_sync();
        uint32_t carry = 0;
        for (uint32_t base = 0; base < nbk; base += 64) {
            const uint32_t i = base + lane;
            const uint32_t v = i < nbk ? cnt[i] : 0u;
            uint32_t x = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (lane >= (uint32_t)o) x += y;
            }
            if (i < nbk) {
                cnt[i] = carry + x - v;
                offs[i] = carry + x - v;
            }
            carry += __shfl(x, 63, 64);
        }
        if (lane == 0) offs[nbk] = m;
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < KPL; j++) {
            if (j * 64 + lane < m) {
                const uint32_t pos = atomicAdd(&cnt[bkt[j]], 1u);
                a.tkeys[kb + pos] = key[j];
                if (spays_all) a.tpays[kb + pos] = pay[j];
            }
        }
        wave_lds_sync();
    }
}

// Block-wide in-place exclusive scan of arr[0..len) (LDS or global via pointer
// kind); also writes the result to out[0..len) and out[len] = total.
template <typename LoadF, typename StoreF>
__device__ __forceinline__ void block_scan_array(uint32_t len, LoadF ld, StoreF st, uint32_t* tmp) {
    uint32_t carry = 0;
    for (uint32_t base = 0; base < len; base += kBlock) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < len ? ld(i) : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan(v, tmp, total);
        if (i < len) st(i, carry + ex);
        carry += total;
    }
}

// One workgroup per partition of biglist (bucket arrays beyond a wave's LDS
// slice): LDS counters up to ocap buckets, global atomics beyond.
template <int HK>
__global__ __launch_bounds__(kBlock) void k_build_big(BuildArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* tmp = reinterpret_cast<uint32_t*>(smem);        // 16 words
    uint32_t* lcnt = tmp + 16;                                // ocap words
    const uint32_t nbig = *a.bigcount;
    for (uint32_t bi = blockIdx.x; bi < nbig; bi += gridDim.x) {
        const uint32_t p = a.biglist[bi];
        const uint32_t kb = a.tkb[p], m = a.tkb[p + 1] - kb;
        const uint32_t ob = a.tob[p], nbk = a.tob[p + 1] - ob - 1;
        uint32_t* offs = a.toffs + ob;
        if (m == 0) {
            for (uint32_t i = threadIdx.x; i <= nbk; i += kBlock) offs[i] = 0;
            continue;
        }
        const bool in_lds = (nbk <= a.ocap);   // (m > 0 here)
        uint32_t* cnt = in_lds ? lcnt : (a.gcursor + ob);
        for (uint32_t i = threadIdx.x; i < nbk; i += kBlock) {
            if (in_lds) cnt[i] = 0;
            else __hip_atomic_store(&cnt[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        // count
        for (uint32_t g = 0; g < a.L.nseg; g++) {
            const Seg& S = a.L.seg[g];
            const uint32_t lo = S.bounds[p], c = S.bounds[p + 1] - lo;
            for (uint32_t i = threadIdx.x; i < c; i += kBlock) {
                const uint32_t b = bucket_of(hash64<HK>(static_cast<uint64_t>(S.keys[lo + i]), a.seed), nbk);
                if (in_lds) atomicAdd(&cnt[b], 1u);
                else __hip_atomic_fetch_add(&cnt[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        // bucket offsets (exclusive), cursors = offsets
        if (in_lds) {
            block_scan_array(
                nbk, [&](uint32_t i) { return cnt[i]; },
                [&](uint32_t i, uint32_t v) {
                    cnt[i] = v;
                    offs[i] = v;
                },
                tmp);
        } else {
            block_scan_array(
                nbk,
                [&](uint32_t i) {
                    return __hip_atomic_load(&cnt[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                },
                [&](uint32_t i, uint32_t v) {
                    __hip_atomic_store(&cnt[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    offs[i] = v;
                },
                tmp);
        }
        if (threadIdx.x == 0) offs[nbk] = m;
        __syncthreads();
        // scatter into bucket order
        for (uint32_t g = 0; g < a.L.nseg; g++) {
            const Seg& S = a.L.seg[g];
            const uint32_t lo = S.bounds[p], c = S.bounds[p + 1] - lo;
            for (uint32_t i = threadIdx.x; i < c; i += kBlock) {
                const int64_t key = S.keys[lo + i];
                const int64_t pay = S.pays ? S.pays[lo + i] : 0;
                const uint64_t h = hash64<HK>(static_cast<uint64_t>(key), a.seed);
                const uint32_t b = bucket_of(h, nbk);
                uint32_t pos;
                if (in_lds) pos = atomicAdd(&cnt[b], 1u);
                else pos = __hip_atomic_fetch_add(&cnt[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                a.tkeys[kb + pos] = key;
                if (S.pays) a.tpays[kb + pos] = pay;
            }
        }
        __syncthreads();
    }
}

struct ProbeArgs {
    const int64_t* skeys;
    const int64_t* tkeys;
    const uint32_t* toffs;
    const ProbeItem* items;
    const uint32_t* nitems;   // device scalar (itb[P])
    unsigned long long* count;
    uint64_t seed;
};

// Probe ITEMS keys per lane in phases so the table reads of all keys are in
// flight together: bucket bounds, then each bucket's first key, then (rarely)
// the rest of a bucket. A key counts once (first match, LinearProbing.hpp:160-180).
// Key j of this lane is item key j * STRIDE + idx (idx: thread or lane index).
template <int HK, int ITEMS, int STRIDE = kBlock, typename KP, typename OP>
__device__ __forceinline__ uint32_t probe_keys(const int64_t (&k)[ITEMS], uint32_t valid_n,
                                               KP K, OP O, uint32_t nbk, uint64_t seed,
                                               uint32_t idx = threadIdx.x) {
    uint32_t lo[ITEMS], hi[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const bool v = static_cast<uint32_t>(j * STRIDE) + idx < valid_n;
        const uint32_t b = bucket_of(hash64<HK>(static_cast<uint64_t>(k[j]), seed), nbk);
        lo[j] = v ? O[b] : 0u;
        hi[j] = v ? O[b + 1] : 0u;
    }
    uint32_t hits = 0;
    bool more = false;
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const bool nonempty = lo[j] < hi[j];
        const bool hit = nonempty && K[nonempty ? lo[j] : 0] == k[j];
        hits += hit;
        lo[j] = hit ? hi[j] : lo[j] + 1;   // consumed
        more |= lo[j] < hi[j];
    }
    if (more) {
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            for (uint32_t t = lo[j]; t < hi[j]; t++) {
                if (K[t] == k[j]) {
                    hits++;
                    break;
                }
            }
        }
    }
    return hits;
}

// probe_keys returning one bit per key (bit j: key j of this lane matched).
template <int HK, int ITEMS, typename KP, typename OP>
__device__ __forceinline__ uint32_t probe_bits(const int64_t (&k)[ITEMS], uint32_t valid_n, KP K, OP O,
                                               uint32_t nbk, uint64_t seed, uint32_t lane) {
    uint32_t lo[ITEMS], hi[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const bool v = static_cast<uint32_t>(j * 64) + lane < valid_n;
        const uint32_t b = bucket_of(hash64<HK>(static_cast<uint64_t>(k[j]), seed), nbk);
        lo[j] = v ? O[b] : 0u;
        hi[j] = v ? O[b + 1] : 0u;
    }
    uint32_t bits = 0;
    bool more = false;
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const bool nonempty = lo[j] < hi[j];
        const bool hit = nonempty && K[nonempty ? lo[j] : 0] == k[j];
        bits |= static_cast<uint32_t>(hit) << j;
        lo[j] = hit ? hi[j] : lo[j] + 1;
        more |= lo[j] < hi[j];
    }
    if (more) {
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            for (uint32_t t = lo[j]; t < hi[j]; t++) {
                if (K[t] == k[j]) {
                    bits |= 1u << j;
                    break;
                }
            }
        }
    }
    return bits;
}

__device__ __forceinline__ ProbeItem load_item(const ProbeItem* items, uint32_t i, uint32_t n) {
    ProbeItem it{};
    if (i < n) {
        const uint4* q = reinterpret_cast<const uint4*>(items + i);
        const uint4 x = q[0], y = q[1];
        it.s_lo = x.x;
        it.s_cnt = x.y;
        it.kb = x.z;
        it.m = x.w;
        it.ob = y.x;
        it.nbk = y.y;
    }
    return it;
}

// Persistent probe over work items, software-pipelined one item deep: while
// item i is probed from LDS, item i+1's S keys and table slice (KPT keys and
// OPT bucket offsets per lane) are already in flight into registers, and the
// descriptor of item i+2 is being fetched. Tables larger than the LDS slice
// (KPT * 256 keys) are probed in place from global memory (L2-resident).
template <int HK, int ITEMS, int KPT>
__global__ __launch_bounds__(kBlock) void k_probe(ProbeArgs a) {
    constexpr uint32_t KCAP = kBlock * KPT;        // staged table keys
    constexpr int OPT = KPT / 2 + 1;               // staged bucket offsets per lane
    constexpr uint32_t OCAP = kBlock * OPT;
    __shared__ int64_t lk[KCAP];
    __shared__ uint32_t lo[OCAP];
    __shared__ uint32_t red[kWaves];
    const uint32_t n = *a.nitems;
    const uint32_t G = gridDim.x, tid = threadIdx.x;
    uint32_t hits = 0;

    uint32_t item = blockIdx.x;
    ProbeItem cur = load_item(a.items, item, n);
    ProbeItem nxt = load_item(a.items, item + G, n);
    int64_t k[ITEMS], tk[KPT];
    uint32_t to[OPT];
    auto fetch = [&](const ProbeItem& it, int64_t (&kk)[ITEMS], int64_t (&tkk)[KPT], uint32_t (&too)[OPT]) {
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t off = j * kBlock + tid;
            kk[j] = off < it.s_cnt ? a.skeys[it.s_lo + off] : 0;
        }
        const bool stage = it.m <= KCAP && it.nbk + 1 <= OCAP;
#pragma unroll
        for (int j = 0; j < KPT; j++) {
            const uint32_t i = j * kBlock + tid;
            tkk[j] = (stage && i < it.m) ? a.tkeys[it.kb + i] : 0;
        }
#pragma unroll
        for (int j = 0; j < OPT; j++) {
            const uint32_t i = j * kBlock + tid;
            too[j] = (stage && i <= it.nbk) ? a.toffs[it.ob + i] : 0u;
        }
    };
    if (item < n) fetch(cur, k, tk, to);
    for (; item < n; item += G) {
        const bool stage = cur.m <= KCAP && cur.nbk + 1 <= OCAP;
        if (stage) {
#pragma unroll
            for (int j = 0; j < KPT; j++) {
                const uint32_t i = j * kBlock + tid;
                if (i < cur.m) lk[i] = tk[j];
            }
#pragma unroll
            for (int j = 0; j < OPT; j++) {
                const uint32_t i = j * kBlock + tid;
                if (i <= cur.nbk) lo[i] = to[j];
            }
        }
        __syncthreads();
        // keep the probe keys of this item; start the next item's loads
        int64_t kc[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) kc[j] = k[j];
        const ProbeItem nn = load_item(a.items, item + 2 * G, n);
        if (item + G < n) fetch(nxt, k, tk, to);
        if (stage) {
            hits += probe_keys<HK, ITEMS>(kc, cur.s_cnt, lk, lo, cur.nbk, a.seed);
        } else {
            hits += probe_keys<HK, ITEMS>(kc, cur.s_cnt, a.tkeys + cur.kb, a.toffs + cur.ob, cur.nbk, a.seed);
        }
        __syncthreads();
        cur = nxt;
        nxt = nn;
    }
    // block reduce -> one atomic per workgroup
    uint32_t x = hits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = x;
    __syncthreads();
    if (tid == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kWaves; w++) t += red[w];
        if (t) atomicAdd(a.count, t);
    }
}

// Persistent probe with one WAVE per work item (S chunks of <= 64 * KPL keys):
// each wave stages its item's table (<= TCAP keys, <= TCAP / 2 + 1 bucket
// offsets) into its own LDS slice and probes from there, ordered by the wave's
// own in-order LDS queue: no workgroup barriers, so small items (the
// multi-GPU case: |S| / (W * P) keys per partition) cost no block-wide
// synchronisation. The next item's S keys, table keys and offsets are loaded
// into registers while the current one is probed. Tables beyond the slice
// are probed in place from global memory.
template <int HK, int KPL, int TCAP>
__global__ __launch_bounds__(kBlock) void k_probe_wave(ProbeArgs a) {
    constexpr int TPL = TCAP / 64;              // staged table keys per lane
    constexpr int OCAP = TCAP / 2 + 1;          // table_buckets(TCAP) + 1
    constexpr int OPL = (OCAP + 63) / 64;       // staged offsets per lane
    __shared__ int64_t lk_all[kWaves][TCAP];
    __shared__ uint32_t lo_all[kWaves][OPL * 64];
    __shared__ uint32_t red[kWaves];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int64_t* lk = lk_all[wave];
    uint32_t* lo = lo_all[wave];
    const uint32_t n = *a.nitems;
    const uint32_t W = gridDim.x * kWaves;
    uint32_t hits = 0;

    uint32_t item = blockIdx.x * kWaves + wave;
    ProbeItem cur = load_item(a.items, item, n);
    int64_t k[KPL], tk[TPL];
    uint32_t to[OPL];
    auto fetch = [&](const ProbeItem& it, int64_t (&kk)[KPL], int64_t (&tkk)[TPL], uint32_t (&too)[OPL]) {
#pragma unroll
        for (int j = 0; j < KPL; j++) {
            const uint32_t off = j * 64 + lane;
            kk[j] = off < it.s_cnt ? a.skeys[it.s_lo + off] : 0;
        }
        const bool stage = it.m <= static_cast<uint32_t>(TCAP) && it.nbk + 1 <= static_cast<uint32_t>(OCAP);
#pragma unroll
        for (int j = 0; j < TPL; j++) {
            const uint32_t i = j * 64 + lane;
            tkk[j] = (stage && i < it.m) ? a.tkeys[it.kb + i] : 0;
        }
#pragma unroll
        for (int j = 0; j < OPL; j++) {
            const uint32_t i = j * 64 + lane;
            too[j] = (stage && i <= it.nbk) ? a.toffs[it.ob + i] : 0u;
        }
    };
    if (item < n) fetch(cur, k, tk, to);
    for (; item < n; item += W) {
        const bool stage = cur.m <= static_cast<uint32_t>(TCAP) && cur.nbk + 1 <= static_cast<uint32_t>(OCAP);
        if (stage) {
#pragma unroll
            for (int j = 0; j < TPL; j++) {
                const uint32_t i = j * 64 + lane;
                if (i < cur.m) lk[i] = tk[j];
            }
#pragma unroll
            for (int j = 0; j < OPL; j++) {
                const uint32_t i = j * 64 + lane;
                if (i <= cur.nbk) lo[i] = to[j];
            }
        }
        wave_lds_sync();
        int64_t kc[KPL];
#pragma unroll
        for (int j = 0; j < KPL; j++) kc[j] = k[j];
        const ProbeItem nxt = load_item(a.items, item + W, n);
        if (item + W < n) fetch(nxt, k, tk, to);
        if (stage)
            hits += probe_keys<HK, KPL, 64>(kc, cur.s_cnt, lk, lo, cur.nbk, a.seed, lane);
        else
            hits += probe_keys<HK, KPL, 64>(kc, cur.s_cnt, a.tkeys + cur.kb, a.toffs + cur.ob, cur.nbk, a.seed, lane);
        wave_lds_sync();   // this item's LDS reads before the next item's stores
        cur = nxt;
    }
    uint32_t x = hits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if (lane == 0) red[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kWaves; w++) t += red[w];
        if (t) atomicAdd(a.count, t);
    }
}

// ---------------------------------------------------------------------------
// Fused per-partition join (the reference's Join() loop, RadixCluster/
// HashJoin.hpp:267-303: for each partition, build its hash table, then probe
// it) with the table in LDS: it never goes to HBM.
//
// Work items: partition p's S keys in chunks of <= kFusedChunk; item slots
// have the closed form itb[p] = floor(sb[p] / kFusedChunk) + p (enough slots
// for ceil(s_p / chunk) items; the rest are empty), so no scan is needed.
// One WAVE per item: R_p is gathered from the build segments (lane g loads
// segment g's bounds, a wave prefix maps flat indices to rows), hashed and
// counting-sorted into a bucketed table in the wave's LDS slice (<= TCAP keys
// per round), then the item's S keys are probed 64 * KPL at a time. A
// partition with more than TCAP build tuples is joined in rounds of TCAP,
// keeping one hit bit per S key of the item (semi-join: a key counts once).
// ---------------------------------------------------------------------------
constexpr uint32_t kFusedChunk = 4096;   // S keys per item (16 probe rounds of 64 x 4)
constexpr int kFusedKPL = 4;             // S keys per lane per probe round
constexpr int kFusedTcap = 256;          // build keys per LDS table round

struct FusedItem {
    uint32_t s_lo, s_cnt, p, pad;
};

// One wave per partition writes its item slots [itb[p], itb[p+1]).
__global__ __launch_bounds__(kBlock) void k_fused_items(const uint32_t* sbounds, uint32_t P, FusedItem* items) {
    const uint32_t p = blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (p >= P) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t sb = sbounds[p], se = sbounds[p + 1];
    const uint32_t lo = sb / kFusedChunk + p, hi = se / kFusedChunk + p + 1;
    for (uint32_t i = lo + lane; i < hi; i += 64) {
        FusedItem it;
        const uint32_t s0 = sb + (i - lo) * kFusedChunk;
        it.s_lo = s0;
        it.s_cnt = s0 < se ? min(kFusedChunk, se - s0) : 0u;
        it.p = p;
        it.pad = 0;
        items[i] = it;
    }
}

struct FusedArgs {
    SegList L;
    const int64_t* skeys;
    const uint32_t* sbounds;
    const FusedItem* items;
    uint32_t nitems;
    uint32_t pad;
    unsigned long long* count;
    unsigned long long* cycles;   // [0] build, [1] probe: wave clock sums (time split)
    uint64_t seed;
};

template <int KPL>
__device__ __forceinline__ void fused_load_s(const int64_t* skeys, uint32_t lo, uint32_t n, uint32_t lane,
                                             int64_t (&k)[KPL]) {
#pragma unroll
    for (int j = 0; j < KPL; j++) {
        const uint32_t off = j * 64 + lane;
        k[j] = off < n ? skeys[lo + off] : 0;
    }
}

// Latency schedule per wave: the next item's descriptor is fetched one item
// ahead; an item's first S sub-chunk is loaded together with its R bounds and
// R keys; sub-chunk k + 1 is loaded while k is probed.
// 5 waves per SIMD at KPL = 4 (92 VGPRs, no spill): the S loads in flight
// per CU, not the arithmetic, bound this kernel
template <int HK, int KPL, int TCAP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KPL <= 2 ? 6 : (KPL <= 4 ? 5 : 3), 8))) void k_join_fused(
    FusedArgs a) {
    constexpr int RPL = TCAP / 64;                 // build keys per lane per round
    constexpr int OCAP = TCAP / 2 + 1;             // bucket offsets (table_buckets(TCAP) + 1)
    constexpr uint32_t SUB = 64 * KPL;             // S keys per probe sub-chunk
    constexpr int NSUB = kFusedChunk / SUB;        // sub-chunks per item (hit bits: NSUB * KPL <= 64)
    static_assert(NSUB * KPL <= 64, "hit bits per lane");
    __shared__ int64_t lk_all[kWaves][TCAP];
    __shared__ uint32_t lo_all[kWaves][OCAP];
    __shared__ uint32_t cur_all[kWaves][OCAP];
    __shared__ unsigned long long red[kWaves][3];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int64_t* lk = lk_all[wave];
    uint32_t* loffs = lo_all[wave];   // bucket starts, [nbk] = keys of the round
    uint32_t* lcur = cur_all[wave];   // counts, then placement cursors
    const uint32_t nseg = a.L.nseg;
    const int64_t* segk = lane < nseg ? a.L.seg[lane].keys : nullptr;
    const uint32_t* segb = lane < nseg ? a.L.seg[lane].bounds : nullptr;
    const uint32_t W = gridDim.x * kWaves;
    unsigned long long hits = 0, cyc_b = 0, cyc_p = 0;

    uint32_t item = blockIdx.x * kWaves + wave;
    FusedItem it = item < a.nitems ? a.items[item] : FusedItem{0, 0, 0, 0};
    for (; item < a.nitems; item += W) {
        const FusedItem nxt = item + W < a.nitems ? a.items[item + W] : FusedItem{0, 0, 0, 0};
        if (it.s_cnt == 0) {
            it = nxt;
            continue;
        }
        const uint64_t tb0 = wall_clock64();
        const uint32_t p = it.p;
        uint32_t rlo = 0, rc = 0;
        if (lane < nseg) {
            rlo = segb[p];
            rc = segb[p + 1] - rlo;
        }
        int64_t sk[KPL];
        fused_load_s<KPL>(a.skeys, it.s_lo, min(SUB, it.s_cnt), lane, sk);
        uint32_t inc = rc;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= static_cast<uint32_t>(o)) inc += y;
        }
        const uint32_t m = __shfl(inc, static_cast<int>(nseg - 1), 64);
        if (m == 0) {   // empty build partition: no S key of p matches
            it = nxt;
            continue;
        }
        const int64_t rowoff = static_cast<int64_t>(rlo) - static_cast<int64_t>(inc - rc);
        const uint32_t nsub = (it.s_cnt + SUB - 1) / SUB;
        uint64_t hitbits = 0;   // bit (sub * KPL + j): S key j of sub-chunk sub matched
        for (uint32_t rb = 0; rb < m; rb += TCAP) {
            const uint64_t tb = rb == 0 ? tb0 : wall_clock64();
            const uint32_t mr = min(static_cast<uint32_t>(TCAP), m - rb);
            const uint32_t nbk = table_buckets(mr);
            const uint32_t rj = (mr + 63) / 64;   // rounds of 64 build keys in use
            int64_t rk[RPL];
            uint32_t bk[RPL];
            if (nseg == 1) {   // one build segment (single GPU): plain strided loads
                const int64_t* kp = a.L.seg[0].keys + __builtin_amdgcn_readfirstlane(rlo);
#pragma unroll
                for (int j = 0; j < RPL; j++) {
                    const uint32_t f = rb + j * 64 + lane;
                    rk[j] = (static_cast<uint32_t>(j) < rj && j * 64 + lane < mr) ? kp[f] : 0;
                }
            } else
#pragma unroll
            for (int j = 0; j < RPL; j++) {
                rk[j] = 0;
                if (static_cast<uint32_t>(j) < rj) {
                    const uint32_t f = rb + j * 64 + lane;
                    uint32_t g = 0;
                    for (uint32_t l = 0; l + 1 < nseg; l++)
                        g += f >= static_cast<uint32_t>(__shfl(inc, l, 64)) ? 1u : 0u;
                    const int64_t ro = __shfl(rowoff, static_cast<int>(g), 64);
                    const int64_t* kp = reinterpret_cast<const int64_t*>(
                        __shfl(reinterpret_cast<intptr_t>(segk), static_cast<int>(g), 64));
                    if (j * 64 + lane < mr) rk[j] = kp[static_cast<int64_t>(f) + ro];
                }
            }
            for (uint32_t i = lane; i < nbk; i += 64) lcur[i] = 0;
            wave_lds_sync();
#pragma unroll
            for (int j = 0; j < RPL; j++) {
                if (static_cast<uint32_t>(j) < rj) {
                    bk[j] = bucket_of(hash64<HK>(static_cast<uint64_t>(rk[j]), a.seed), nbk);
                    if (j * 64 + lane < mr) atomicAdd(&lcur[bk[j]], 1u);
                }
            }
            wave_lds_sync();
            // exclusive scan: bucket starts (loffs[0..nbk]) and placement cursors
            uint32_t carry = 0;
            for (uint32_t base = 0; base < nbk; base += 64) {
                const uint32_t i = base + lane;
                const uint32_t v = i < nbk ? lcur[i] : 0u;
                uint32_t x = v;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(x, o, 64);
                    if (lane >= static_cast<uint32_t>(o)) x += y;
                }
                if (i < nbk) {
                    loffs[i] = carry + x - v;
                    lcur[i] = carry + x - v;
                }
                carry += __shfl(x, 63, 64);
            }
            if (lane == 0) loffs[nbk] = mr;
            wave_lds_sync();
#pragma unroll
            for (int j = 0; j < RPL; j++) {
                if (static_cast<uint32_t>(j) < rj && j * 64 + lane < mr) lk[atomicAdd(&lcur[bk[j]], 1u)] = rk[j];
            }
            wave_lds_sync();
            const uint64_t tp = wall_clock64();
            cyc_b += tp - tb;
            // probe the item's S sub-chunks; sub-chunk 0 is already in registers
            // (reloaded for later rounds of an oversized build partition)
            if (rb > 0) fused_load_s<KPL>(a.skeys, it.s_lo, min(SUB, it.s_cnt), lane, sk);
            for (uint32_t sub = 0; sub < nsub; sub++) {
                int64_t nk[KPL];
                if (sub + 1 < nsub)
                    fused_load_s<KPL>(a.skeys, it.s_lo + (sub + 1) * SUB, min(SUB, it.s_cnt - (sub + 1) * SUB), lane, nk);
                const uint32_t n_sub = min(SUB, it.s_cnt - sub * SUB);
                hitbits |= static_cast<uint64_t>(probe_bits<HK, KPL>(sk, n_sub, lk, loffs, nbk, a.seed, lane))
                           << (sub * KPL);
                if (sub + 1 < nsub) {
#pragma unroll
                    for (int j = 0; j < KPL; j++) sk[j] = nk[j];
                }
            }
            wave_lds_sync();   // this round's LDS reads before the next round's stores
            cyc_p += wall_clock64() - tp;
        }
        hits += __popcll(hitbits);
        it = nxt;
    }
    unsigned long long x = hits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if (lane == 0) {
        red[wave][0] = x;
        red[wave][1] = cyc_b;
        red[wave][2] = cyc_p;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0, b = 0, q = 0;
        for (int w = 0; w < kWaves; w++) {
            t += red[w][0];
            b += red[w][1];
            q += red[w][2];
        }
        if (t) atomicAdd(a.count, t);
        atomicAdd(&a.cycles[0], b);
        atomicAdd(&a.cycles[1], q);
    }
}

// ---------------------------------------------------------------------------
// NoPartitioning: global bucketized linear probing.
// ---------------------------------------------------------------------------
constexpr int kNPSlots = 7;

struct alignas(64) NPBucket {
    int64_t key[kNPSlots];
    uint32_t fill;   // claimed slots; > 7 once full (readers clamp)
    uint32_t pad;
};

__device__ __forceinline__ uint32_t np_home(uint64_t h, uint32_t nb) {
    return static_cast<uint32_t>(((h >> 32) * static_cast<uint64_t>(nb)) >> 32);
}

// Region layout of the NoPartitioning table (the default build): the table is
// 2^rbits regions of nbr buckets; a key's region is the low rbits of its hash
// (exactly the radix partition q = h & (2^rbits - 1)) and its home bucket
// inside the region comes from the high 32 bits. Linear probing still walks
// b, b + 1, ... over the whole table, so a full last bucket of a region
// continues in the next region.
struct NPHome {
    uint32_t nb, nbr, rbits, pad;
};

__device__ __forceinline__ uint32_t np_home_r(uint64_t h, const NPHome& g) {
    if (g.rbits == 0) return np_home(h, g.nb);
    const uint32_t r = static_cast<uint32_t>(h) & ((1u << g.rbits) - 1);
    return r * g.nbr + static_cast<uint32_t>(((h >> 32) * static_cast<uint64_t>(g.nbr)) >> 32);
}

// Region build: R radix-partitioned on q = h & (2^rbits - 1) beforehand
// (partition_side), one workgroup per region builds that region's buckets in
// LDS (LDS atomics claim slots; no device-scope atomics, which on MI355X go
// to the memory side: the atomic build runs at ~14 G inserts/s) and writes the
// region out as whole 64-B buckets. A tuple that walks past the region's last
// bucket goes to an overflow list, inserted afterwards by k_np_build_overflow
// from the next region's first bucket (the probe walks the same way).
// LDS: nbr * (4 + 56) bytes.
template <int HK>
__global__ __launch_bounds__(kBlock) void k_np_build_region(const int64_t* keys, const int64_t* pays_in,
                                                            const uint32_t* bounds, NPHome g, NPBucket* tab,
                                                            int64_t* pays, uint64_t seed, uint32_t* ovf_n,
                                                            longlong2* ovf, uint32_t* ovf_b) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t nbr = g.nbr, r = blockIdx.x;
    int64_t* lkey = reinterpret_cast<int64_t*>(smem);
    uint32_t* lfill = reinterpret_cast<uint32_t*>(lkey + static_cast<size_t>(nbr) * kNPSlots);
    for (uint32_t i = threadIdx.x; i < nbr * kNPSlots; i += kBlock) lkey[i] = 0;
    for (uint32_t i = threadIdx.x; i < nbr; i += kBlock) lfill[i] = 0;
    __syncthreads();
    const uint32_t lo = bounds[r], hi = bounds[r + 1];
    const size_t b0 = static_cast<size_t>(r) * nbr;
    // 4 tuples per thread per round: their loads and hashes before the LDS claims
    constexpr int IT = 4;
    for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += IT * kBlock) {
        int64_t k[IT], v[IT];
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint32_t i = i0 + j * kBlock;
            k[j] = i < hi ? keys[i] : 0;
            v[j] = i < hi ? pays_in[i] : 0;
        }
#pragma unroll
        for (int j = 0; j < IT; j++) {
            if (i0 + j * kBlock >= hi) break;
            const uint64_t h = hash64<HK>(static_cast<uint64_t>(k[j]), seed);
            uint32_t b = static_cast<uint32_t>(((h >> 32) * static_cast<uint64_t>(nbr)) >> 32);
            for (;;) {
                const uint32_t slot = atomicAdd(&lfill[b], 1u);
                if (slot < kNPSlots) {
                    lkey[b * kNPSlots + slot] = k[j];
                    pays[(b0 + b) * kNPSlots + slot] = v[j];
                    break;
                }
                if (++b == nbr) {   // past the region: insert later from the next region
                    const uint32_t o = atomicAdd(ovf_n, 1u);
                    ovf[o] = make_longlong2(k[j], v[j]);
                    ovf_b[o] = static_cast<uint32_t>((b0 + nbr) % g.nb);
                    break;
                }
            }
        }
    }
    __syncthreads();
    // whole buckets out: 4 lanes per 64-B bucket, consecutive buckets contiguous
    longlong2* out = reinterpret_cast<longlong2*>(tab + b0);
    for (uint32_t i = threadIdx.x; i < nbr * 4; i += kBlock) {
        const uint32_t b = i >> 2, w = i & 3;
        longlong2 v;
        if (w < 3) {
            v = make_longlong2(lkey[b * kNPSlots + 2 * w], lkey[b * kNPSlots + 2 * w + 1]);
        } else {
            v = make_longlong2(lkey[b * kNPSlots + 6], static_cast<int64_t>(lfill[b]));
        }
        out[i] = v;
    }
}

// The overflow list of k_np_build_region, inserted with device atomics (rare:
// about one tuple per few regions at the default 1.25 ratio).
__global__ __launch_bounds__(kBlock) void k_np_build_overflow(const uint32_t* ovf_n, const longlong2* ovf,
                                                              const uint32_t* ovf_b, NPBucket* tab, int64_t* pays,
                                                              uint32_t nb) {
    const uint32_t n = *ovf_n;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const longlong2 t = ovf[i];
        uint32_t b = ovf_b[i];
        for (uint32_t step = 0; step < nb; step++) {
            const uint32_t slot = atomicAdd(&tab[b].fill, 1u);
            if (slot < kNPSlots) {
                tab[b].key[slot] = t.x;
                pays[static_cast<size_t>(b) * kNPSlots + slot] = t.y;
                break;
            }
            b = (b + 1 == nb) ? 0 : b + 1;
        }
    }
}

// One bucketized-linear-probing lookup from home bucket b (NoPartitioning
// semantics, LinearProbing.hpp:160-180: stop at the first non-full bucket).
__device__ __forceinline__ bool np_lookup(const NPBucket* tab, uint32_t nb, uint32_t b, int64_t key) {
    for (uint32_t step = 0; step < nb; step++) {
        const longlong2* bp = reinterpret_cast<const longlong2*>(tab + b);
        const longlong2 q0 = bp[0], q1 = bp[1], q2 = bp[2], q3 = bp[3];
        const uint32_t fill = static_cast<uint32_t>(q3.y);
        const uint32_t c = fill < kNPSlots ? fill : kNPSlots;
        if ((c > 0 && q0.x == key) || (c > 1 && q0.y == key) || (c > 2 && q1.x == key) || (c > 3 && q1.y == key) ||
            (c > 4 && q2.x == key) || (c > 5 && q2.y == key) || (c > 6 && q3.x == key))
            return true;
        if (fill < kNPSlots) return false;
        b = (b + 1 == nb) ? 0 : b + 1;
    }
    return false;
}

// NT: the probe keys are streamed with nontemporal loads, so the 3.2 GB of S
// passing through does not evict the table's hot buckets from L2 / MALL (the
// table is ~114 MB at 10M build tuples; under Zipf most probes hit a few
// thousand buckets).
template <int HK, int ITEMS, int NT>
__global__ __launch_bounds__(kBlock) void k_np_probe(const longlong2* S, uint64_t nS,
                                                     const NPBucket* tab, NPHome g,
                                                     uint64_t seed, unsigned long long* count) {
    const uint32_t nb = g.nb;
    __shared__ uint32_t red[kWaves];
    uint32_t hits = 0;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kBlock * ITEMS;
    for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * kBlock * ITEMS; base < nS; base += stride) {
        int64_t k[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t idx = base + static_cast<uint64_t>(j) * kBlock + threadIdx.x;
            if constexpr (NT > 0)
                k[j] = idx < nS ? __builtin_nontemporal_load(&S[idx].x) : 0;
            else
                k[j] = idx < nS ? S[idx].x : 0;
        }
        // every home bucket of the round is requested before any is compared:
        // ITEMS random 64-B reads in flight per thread, not one
        uint32_t b[ITEMS];
        longlong2 q[ITEMS][4];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            b[j] = np_home_r(hash64<HK>(static_cast<uint64_t>(k[j]), seed), g);
            const longlong2* bp = reinterpret_cast<const longlong2*>(tab + b[j]);
            if constexpr (NT > 1) {
                typedef long long v2i __attribute__((ext_vector_type(2)));
                const v2i* vp = reinterpret_cast<const v2i*>(bp);
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    const v2i a = __builtin_nontemporal_load(vp + w);
                    q[j][w] = make_longlong2(a.x, a.y);
                }
            } else {
#pragma unroll
                for (int w = 0; w < 4; w++) q[j][w] = bp[w];
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t idx = base + static_cast<uint64_t>(j) * kBlock + threadIdx.x;
            if (idx < nS) {
                const int64_t key = k[j];
                const uint32_t fill = static_cast<uint32_t>(q[j][3].y);
                const uint32_t c = fill < kNPSlots ? fill : kNPSlots;
                const bool hit = (c > 0 && q[j][0].x == key) || (c > 1 && q[j][0].y == key) ||
                                 (c > 2 && q[j][1].x == key) || (c > 3 && q[j][1].y == key) ||
                                 (c > 4 && q[j][2].x == key) || (c > 5 && q[j][2].y == key) ||
                                 (c > 6 && q[j][3].x == key);
                if (hit)
                    hits++;
                else if (fill >= kNPSlots)   // full home bucket: continue in the next ones (rare)
                    hits += np_lookup(tab, nb, b[j] + 1 == nb ? 0 : b[j] + 1, key) ? 1u : 0u;
            }
        }
    }
    uint32_t x = hits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kWaves; w++) t += red[w];
        if (t) atomicAdd(count, t);
    }
}

// ---------------------------------------------------------------------------
// Partitioned bucket tables in HBM, for partitions too large for the fused
// LDS join (the reference's small-P configurations, e.g. -p 32: 312K build
// tuples per partition). Partition p owns buckets [tob[p], tob[p+1]) of
// 64-B NoPartitioning buckets (nb_p = ceil(m_p * ratio / 7)); a tuple's
// partition is recomputed from its hash (q = the pass digits concatenated),
// so neither build nor probe needs a work list. S is probed in its
// partitioned order: consecutive lanes hit the same partition's region,
// which stays in L2 while that partition is being probed.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t q_of_hash(uint64_t h, const DigitFn& f) {
    return static_cast<uint32_t>(q_from_hash(h, f));
}

// arr[p] = buckets of partition p (>= 1), arr[P] = 0; exclusive scan -> tob.
__global__ __launch_bounds__(kBlock) void k_pt_prep(SegList L, uint32_t ratio_x256, uint32_t* arr) {
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (p > L.P) return;
    if (p == L.P) {
        arr[p] = 0;
        return;
    }
    uint32_t m = 0;
    for (uint32_t g = 0; g < L.nseg; g++) m += L.seg[g].bounds[p + 1] - L.seg[g].bounds[p];
    const uint64_t slots = (static_cast<uint64_t>(m) * ratio_x256 + 255) / 256;
    arr[p] = static_cast<uint32_t>(max<uint64_t>(1, (slots + kNPSlots - 1) / kNPSlots));
}

struct PtabArgs {
    SegList L;
    uint32_t segoff[kMaxSegs + 1];   // prefix of the segments' tuple counts
    NPBucket* tab;
    int64_t* pays;
    const uint32_t* tob;
    DigitFn f;                       // q of a hash: shift 0, all digit bits
    uint64_t seed;
};

template <int HK>
__global__ __launch_bounds__(kBlock) void k_pt_build(PtabArgs a) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.segoff[a.L.nseg]) return;
    uint32_t g = 0;
    while (i >= a.segoff[g + 1]) g++;
    const uint32_t row = i - a.segoff[g];
    const int64_t key = a.L.seg[g].keys[row];
    const int64_t* sp = a.L.seg[g].pays;
    const int64_t pay = sp ? sp[row] : 0;
    const uint64_t h = hash64<HK>(static_cast<uint64_t>(key), a.seed);
    const uint32_t q = q_of_hash(h, a.f);
    const uint32_t base = a.tob[q], nb = a.tob[q + 1] - base;
    NPBucket* tab = a.tab + base;
    uint32_t b = np_home(h, nb);
    for (uint32_t step = 0; step < nb; step++) {
        const uint32_t slot = atomicAdd(&tab[b].fill, 1u);
        if (slot < kNPSlots) {
            tab[b].key[slot] = key;
            if (sp) a.pays[(static_cast<size_t>(base) + b) * kNPSlots + slot] = pay;
            return;
        }
        b = (b + 1 == nb) ? 0 : b + 1;
    }
}

template <int HK, int ITEMS>
__global__ __launch_bounds__(kBlock) void k_pt_probe(const int64_t* skeys, uint32_t nS, const NPBucket* tab,
                                                     const uint32_t* tob, DigitFn f, uint64_t seed,
                                                     unsigned long long* count) {
    __shared__ uint32_t red[kWaves];
    uint32_t hits = 0;
    const uint32_t base0 = blockIdx.x * kBlock * ITEMS;
    int64_t k[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint32_t idx = base0 + j * kBlock + threadIdx.x;
        k[j] = idx < nS ? skeys[idx] : 0;
    }
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const uint32_t idx = base0 + j * kBlock + threadIdx.x;
        if (idx < nS) {
            const uint64_t h = hash64<HK>(static_cast<uint64_t>(k[j]), seed);
            const uint32_t q = q_of_hash(h, f);
            const uint32_t b0 = tob[q], nb = tob[q + 1] - b0;
            hits += np_lookup(tab + b0, nb, np_home(h, nb), k[j]) ? 1u : 0u;
        }
    }
    uint32_t x = hits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kWaves; w++) t += red[w];
        if (t) atomicAdd(count, t);
    }
}

// ---------------------------------------------------------------------------
// Generators and utilities.
// ---------------------------------------------------------------------------
constexpr uint32_t kGenBatch = 4096;

// Rows [first, first + n) of Sequential::FillTable: id = start + i, payload = i (global i).
__global__ __launch_bounds__(kBlock) void k_gen_sequential(longlong2* out, uint64_t n, int64_t start,
                                                           uint64_t first) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kBlock;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
        const int64_t g = static_cast<int64_t>(first + i);
        out[i] = make_longlong2(start + g, g);
    }
}

__device__ __forceinline__ double lcg_next(int64_t& st) {
    const int64_t a = 16807, q = 127773, r = 2836, m = 2147483647LL;
    const int64_t xn = a * (st % q) - r * (st / q);
    st = xn > 0 ? xn : xn + m;
    return static_cast<double>(st) / static_cast<double>(m);
}

// Thread per 4096-tuple batch; Zipf::generate (Zipf.cpp:14-56) per sample.
// Writes global rows [first, first + n) to out[0, n). Bit-exact with the host
// generator: glibc's pow (phj_pow.h) and no contracted arithmetic (the
// reference's x86-64 build has no FMA), so every sample and every batch's LCG
// stream equal the host's.
__global__ __launch_bounds__(kBlock) void k_gen_zipf(longlong2* out, uint64_t n, double alpha,
                                                     uint64_t card, int64_t correction,
                                                     uint64_t seed, uint64_t first) {
#pragma clang fp contract(off)
    using glibc_pow::pow;
    const uint64_t b = first / kGenBatch + static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const uint64_t lo = b * kGenBatch;
    const uint64_t end = first + n;
    if (lo >= end) return;
    const uint64_t hi = lo + kGenBatch < end ? lo + kGenBatch : end;
    const uint64_t M = 2147483646ULL;
    int64_t st = static_cast<int64_t>(1 + (((seed % M) * 1000003ULL + b) % M));
    double skew = 1.001 - alpha;
    const double diff = 1.0 - alpha;
    if (fabs(diff) < 0.01) {
        skew = 0.01 * ((diff < 0) ? 1 : -1);
        alpha = 1.0 - skew;
    }
    const double norm = (pow(static_cast<double>(card), skew) - alpha) / skew;
    for (uint64_t i = lo; i < hi; i++) {
        double sample;
        for (;;) {
            const double u1 = lcg_next(st);
            const double u2 = lcg_next(st);
            double inv;
            if (u1 * norm <= 1.0) inv = u1 * norm;
            else inv = pow((u1 * norm) * skew + alpha, 1.0 / skew);
            sample = floor(inv + 1);
            const double d_orig = pow(sample, -alpha);
            const double d_samp = sample <= 1.0 ? 1.0 / norm : pow(inv, -alpha) / norm;
            if (u2 < d_orig / (d_samp * norm)) break;
        }
        if (i >= first)
            out[i - first] = make_longlong2(static_cast<int64_t>(static_cast<uint64_t>(sample)) + correction,
                                            static_cast<int64_t>(i));
    }
}

__global__ __launch_bounds__(kBlock) void k_count_range(const longlong2* rel, uint64_t n, int64_t lo,
                                                        int64_t hi, unsigned long long* count) {
    __shared__ uint32_t red[kWaves];
    uint32_t c = 0;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kBlock;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
        const int64_t k = rel[i].x;
        c += (k >= lo && k <= hi) ? 1u : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kWaves; w++) t += red[w];
        if (t) atomicAdd(count, t);
    }
}

template <int HK>
__global__ __launch_bounds__(kBlock) void k_hash_keys(const int64_t* keys, uint64_t n, uint64_t seed,
                                                      uint64_t* out) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i < n) out[i] = hash64<HK>(static_cast<uint64_t>(keys[i]), seed);
}

}  // namespace phj
