// phj_cluster.h — the counting radix join with LDS-resident cluster tables.
//
// The reference joins partition by partition: build a LinearProbing table on
// R_p, probe it with S_p, count the S tuples whose Get() finds a key
// (src/RadixCluster/HashJoin.hpp:267-303; Get() = first match,
// src/HashTables/LinearProbing.hpp:160-180). Its partitions are sized so the
// table stays in a CPU cache; here they are sized so the table fits a
// workgroup's LDS (the MI355X's 160 KB per CU):
//
//   pass 1 (both sides): hash codes c = h(k) partitioned into K clusters, the
//     top log2 K bits of the plan's partition number q (so every cluster is a
//     union of whole final partitions of the requested radix / h % P plan);
//     S by the chunked keys-only pass (k_chunk_codes), R by k_hist + scan +
//     k_scatter_codes (codes contiguous per cluster).
//   probe (k_cluster_probe): persistent; workgroup w walks a contiguous range
//     of S's pass-1 tiles (cluster-major). When the cluster changes it builds
//     that cluster's R codes into an open-addressed table in LDS (the R run of
//     ~5-10K codes is read once per workgroup that needs it), then every S code
//     of the tile reads one 16-B bucket in LDS. Nothing but S's codes streams
//     from HBM: no table in HBM, no d2 grouping, no second pass over S.
//
// The final partitions of the plan are never materialised: a cluster's table
// hashes on code bits 24+ (clear of every partition bit), i.e. it is the union
// of its partitions' tables, and the count is the same (equal codes <=> equal
// keys, both hashes being bijections: phj_hash.h).
//
// Table of cluster d: cap slots (a power of two), 2-slot (16-B) buckets,
// home bucket (c >> 24) & (cap / 2 - 1), linear probing over buckets, slot 0
// filled before slot 1, duplicates stored once. An empty slot holds E_d, a code
// of ANOTHER cluster (0 for d != 0: code 0 is in cluster 0; for d = 0 the
// plan's lowest power of two outside cluster 0), so no key value is reserved
// (the reference marks occupancy with a fill counter, LinearProbing.hpp:79-82).
// A cluster with more than `lim` R codes (skewed or adversarial build sides)
// gets its table in HBM instead (k_cluster_big_fill, device atomics; slot
// 4 * B_d + 2 * d, B_d = its first code over all segments: tables never
// overlap), and the probe reads it there: correct for any input, fast for
// the balanced ones.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "phj_hash.h"
#include "phj_partition.h"
#include "phj_table.h"

namespace phj {

constexpr int kClBlock = 1024, kClItems = 4;   // 16 waves, 4 codes per lane: one 4096-slot pass-1 chunk per tile
constexpr uint32_t kClCapMax = 16384;          // LDS table slots (128 KB)
constexpr uint32_t kClCpl = kClCapMax * 3 / 4 / kClBlock;   // R codes per lane at the largest LDS cluster

__host__ __device__ __forceinline__ uint32_t cl_lim(uint32_t cap) { return cap / 4 * 3; }   // load <= 3/4

// HBM table slots of a big cluster of m codes (load <= 2/3, < 3 m + 2 <= 4 m + 2)
__host__ __device__ __forceinline__ uint32_t cl_big_cap(uint32_t m) { return ht_cap_for(m + (m + 1) / 2); }

struct ClusterArgs {
    // S: the chunked keys-only pass 1 (codes), tiles cluster-major
    const int64_t* s_codes;
    const uint32_t* tile_base;    // [nb1 + 1]: tile_base[nb1] = tiles
    const uint32_t* tile_seg;     // tile -> cluster
    const uint32_t* tile_start;   // tile -> first slot
    const uint32_t* tile_cnt;     // tile -> codes
    // R: build segments (one per rank after the all-gather), codes contiguous per cluster
    const int64_t* r_codes[kHtSegs];
    const uint32_t* r_bounds[kHtSegs];   // nb1 + 1 each
    uint32_t nseg, nb1;
    uint32_t cap, lim;            // LDS table slots; clusters of more R codes use the HBM table
    uint64_t e1;                  // E of cluster 0
    uint64_t* gtab;               // HBM tables of the big clusters
    unsigned long long* count;    // {count, failed}
    const uint32_t* err;          // S's pass-1 error word (fold_pass1_error), or null
};

// Cluster d's runs over the segments: sseg[g] = codes before segment g (sseg[nseg] = m),
// sptr[g] = where element r of segment g's run sits, minus r; returns B_d (first code
// over all segments). Wave 0 computes, every thread sees it after the caller's barrier.
__device__ __forceinline__ void cl_runs(const ClusterArgs& a, uint32_t d, uint32_t* sseg, const int64_t** sptr,
                                        uint32_t* sB) {
    const uint32_t tid = threadIdx.x;
    if (tid < 64) {
        uint32_t lo = 0, len = 0;
        if (tid < a.nseg) {
            lo = a.r_bounds[tid][d];
            len = a.r_bounds[tid][d + 1] - lo;
        }
        uint32_t x = len;
#pragma unroll
        for (int o = 1; o < kHtSegs; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (tid >= static_cast<uint32_t>(o)) x += y;
        }
        uint32_t b = lo;
#pragma unroll
        for (int o = 1; o < kHtSegs; o <<= 1) b += __shfl_xor(b, o, 64);
        if (tid < a.nseg) {
            sseg[tid + 1] = x;
            sptr[tid] = a.r_codes[tid] + lo - (x - len);
        }
        if (tid == 0) {
            sseg[0] = 0;
            *sB = b;
        }
    }
}

// Segment of element r of the cluster's run (sseg ascending, nseg <= 16).
__device__ __forceinline__ uint32_t cl_seg_of(const uint32_t* sseg, uint32_t nseg, uint32_t r) {
    uint32_t g = 0;
#pragma unroll
    for (uint32_t step = kHtSegs / 2; step >= 1; step >>= 1)
        if (g + step < nseg && sseg[g + step] <= r) g += step;
    return g;
}

// HBM tables of the clusters beyond the LDS limit: one workgroup per cluster,
// the others return at once (none at the balanced configurations).
__global__ __launch_bounds__(256) void k_cluster_big_fill(ClusterArgs a) {
    __shared__ uint32_t sseg[kHtSegs + 1];
    __shared__ const int64_t* sptr[kHtSegs];
    __shared__ uint32_t sB;
    const uint32_t d = blockIdx.x, tid = threadIdx.x;
    cl_runs(a, d, sseg, sptr, &sB);
    __syncthreads();
    const uint32_t m = sseg[a.nseg];
    if (m <= a.lim) return;   // workgroup-uniform
    const uint64_t e = d == 0 ? a.e1 : 0ull;
    const uint32_t cap = cl_big_cap(m);
    uint64_t* t = a.gtab + 4ull * sB + 2ull * d;
    for (uint32_t sl = tid; sl < cap; sl += 256) t[sl] = e;
    __threadfence();
    __syncthreads();
    for (uint32_t r = tid; r < m; r += 256) {
        const uint32_t g = cl_seg_of(sseg, a.nseg, r);
        ht_insert(t, cap / 2 - 1, e, static_cast<uint64_t>(sptr[g][r]));
    }
}

// The probe. LDS: the cluster table (cap slots) + a few words. PF: tiles
// whose codes are in flight ahead of the one probed (registers: PF * ITEMS codes).
template <int BLOCK, int ITEMS, int PF = 1>
__global__ __launch_bounds__(BLOCK) void k_cluster_probe(ClusterArgs a) {
    constexpr int CPL = kClCapMax * 3 / 4 / BLOCK;   // R codes per lane at the limit
    extern __shared__ __attribute__((aligned(16))) uint64_t tab[];   // [cap]
    __shared__ uint32_t sseg[kHtSegs + 1];
    __shared__ const int64_t* sptr[kHtSegs];
    __shared__ uint32_t sB;
    __shared__ uint32_t red[BLOCK / 64];
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t total = a.tile_base[a.nb1];
    // workgroup -> a contiguous range of tiles; neighbouring ranges on one XCD
    // (they share the cluster at their boundary: its R run is an L2 hit)
    const uint32_t G = gridDim.x, r8 = (blockIdx.x & 7u) * (G >> 3) + (blockIdx.x >> 3);
    const uint32_t t_lo = static_cast<uint32_t>(static_cast<uint64_t>(total) * r8 / G);
    const uint32_t t_hi = static_cast<uint32_t>(static_cast<uint64_t>(total) * (r8 + 1) / G);
    uint32_t hits = 0;
    if (t_lo < t_hi) {   // workgroup-uniform
        int64_t key[PF + 1][ITEMS];   // [0] the tile probed, [1..PF] in flight
        uint32_t vm[PF + 1], dq[PF + 1];
        // tile metadata 64 tiles at a time: lane i holds tile mb + i's {cluster,
        // first slot, codes} (vector loads, read out with readlane: a scalar
        // load per tile would make every later LDS wait -- lgkmcnt covers both
        // -- wait for it too)
        uint32_t mb = 0, mseg = 0, mstart = 0, mcnt = 0;
        auto meta = [&](uint32_t base) {
            mb = base;
            const uint32_t tt = min(base + lane, t_hi - 1);
            mseg = a.tile_seg[tt];
            mstart = a.tile_start[tt];
            mcnt = a.tile_cnt[tt];
        };
        meta(t_lo);
        auto load = [&](uint32_t t, int64_t* k, uint32_t& m, uint32_t& dd) {
            if (t - mb >= 64) meta(t);
            const int idx = static_cast<int>(t - mb);
            dd = __builtin_amdgcn_readlane(mseg, idx);
            const uint32_t lo = __builtin_amdgcn_readlane(mstart, idx), c = __builtin_amdgcn_readlane(mcnt, idx);
            m = 0;
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {   // clamped, unconditional (an empty tile reads slot lo + e)
                const uint32_t e = i * BLOCK + tid;
                k[i] = __builtin_nontemporal_load(a.s_codes + lo + min(e, c - 1u));
                m |= e < c ? (1u << i) : 0u;
            }
        };
#pragma unroll
        for (int f = 0; f < PF; f++) {
            vm[f] = 0;
            dq[f] = 0;
            if (t_lo + f < t_hi) load(t_lo + f, key[f], vm[f], dq[f]);
        }
        uint32_t cur = 0xffffffffu, bmask = 0;
        bool big = false;
        uint64_t e = 0;
        const ulonglong2* tb = reinterpret_cast<const ulonglong2*>(tab);
        for (uint32_t t = t_lo;;) {
            const uint32_t d = dq[0];
            if (d != cur) {   // workgroup-uniform: build cluster d's table
                __syncthreads();   // every probe of the previous table is done
                cl_runs(a, d, sseg, sptr, &sB);
                __syncthreads();
                const uint32_t m = sseg[a.nseg];
                e = d == 0 ? a.e1 : 0ull;
                big = m > a.lim;
                if (!big) {
                    bmask = a.cap / 2 - 1;
                    uint64_t rc[CPL];
#pragma unroll
                    for (int j = 0; j < CPL; j++) {   // every code of the run requested at once
                        const uint32_t r = j * BLOCK + tid;
                        rc[j] = 0;
                        if (r < m) rc[j] = static_cast<uint64_t>(sptr[cl_seg_of(sseg, a.nseg, r)][r]);
                    }
                    ulonglong2* t2 = reinterpret_cast<ulonglong2*>(tab);
                    for (uint32_t b = tid; b <= bmask; b += BLOCK) t2[b] = make_ulonglong2(e, e);
                    __syncthreads();   // cleared
#pragma unroll
                    for (int j = 0; j < CPL; j++) {
                        if (j * BLOCK + tid < m) {
                            const uint64_t c = rc[j];
                            uint32_t b = static_cast<uint32_t>(c >> kHtBucketShift) & bmask;
                            for (;;) {
                                const uint64_t o0 = atomicCAS(reinterpret_cast<unsigned long long*>(&tab[2 * b]), e, c);
                                if (o0 == e || o0 == c) break;
                                const uint64_t o1 = atomicCAS(reinterpret_cast<unsigned long long*>(&tab[2 * b + 1]), e, c);
                                if (o1 == e || o1 == c) break;
                                b = (b + 1) & bmask;
                            }
                        }
                    }
                    __syncthreads();   // built
                } else {
                    bmask = cl_big_cap(m) / 2 - 1;
                }
                cur = d;
            }
            vm[PF] = 0;
            dq[PF] = d;
            if (t + PF < t_hi) load(t + PF, key[PF], vm[PF], dq[PF]);   // workgroup-uniform
            if (!big) {   // LDS: every item's home bucket read, then the walks
                ulonglong2 v[ITEMS];
#pragma unroll
                for (int i = 0; i < ITEMS; i++) v[i] = tb[static_cast<uint32_t>(static_cast<uint64_t>(key[0][i]) >> kHtBucketShift) & bmask];
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    const uint64_t c = static_cast<uint64_t>(key[0][i]);
                    bool hit = v[i].x == c || v[i].y == c;
                    if ((vm[0] >> i) & 1u) {
                        if (!hit && v[i].y != e) {
                            uint32_t b = static_cast<uint32_t>(c >> kHtBucketShift) & bmask;
                            for (;;) {
                                b = (b + 1) & bmask;
                                const ulonglong2 w = tb[b];
                                hit = w.x == c || w.y == c;
                                if (hit || w.y == e) break;
                            }
                        }
                        hits += hit ? 1u : 0u;
                    }
                }
            } else {   // HBM table of a big cluster
                const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(a.gtab + 4ull * sB + 2ull * d);
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    if ((vm[0] >> i) & 1u) {
                        const uint64_t c = static_cast<uint64_t>(key[0][i]);
                        uint32_t b = static_cast<uint32_t>(c >> kHtBucketShift) & bmask;
                        for (;;) {
                            const ulonglong2 w = g2[b];
                            if (w.x == c || w.y == c) {
                                hits++;
                                break;
                            }
                            if (w.y == e) break;
                            b = (b + 1) & bmask;
                        }
                    }
                }
            }
            if (++t >= t_hi) break;
#pragma unroll
            for (int f = 0; f < PF; f++) {
#pragma unroll
                for (int i = 0; i < ITEMS; i++) key[f][i] = key[f + 1][i];
                vm[f] = vm[f + 1];
                dq[f] = dq[f + 1];
            }
        }
    }
    uint32_t x = hits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if (lane == 0) red[wave] = x;
    __syncthreads();
    if (tid == 0) {
        unsigned long long s = 0;
        for (int w = 0; w < BLOCK / 64; w++) s += red[w];
        if (s) atomicAdd(a.count, s);
    }
    fold_pass1_error(a.err, a.count);
}

}  // namespace phj
