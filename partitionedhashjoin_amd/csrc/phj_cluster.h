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
//     S by the chunked keys-only pass (k_chunk_codes_pipe); R by the same
//     pass on one device (its codes read through its pass-1 tile list: "tile
//     mode", below), or by k_hist + scan + k_scatter_codes (codes contiguous
//     per cluster: a multi-GPU member's exchange block, or PHJ_R_CHUNK=0).
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
//
// R's codes of cluster d are "runs": in segment mode one contiguous run per
// build segment g (r_codes[g] + r_bounds[g][d] .. r_bounds[g][d + 1]); in tile
// mode (rt_base set) the cluster's pass-1 tiles [rt_base[d], rt_base[d + 1])
// of R's chunk pool, each a run of rt_cnt codes at rt_start, with
// r_bounds[0] the cluster offsets of R's pass 1 (m and B_d). A cluster whose
// runs exceed kHtSegs (only possible above the LDS limit when R's pass 1 has
// <= 8 shards: <= 8 + lim / 4096 runs below it) takes the HBM table.
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
    unsigned long long* split;    // null, or {build, probe}: the workgroups' wall clocks spent building tables / probing
    unsigned long long* prof;     // PROF kernels: the builds' sections (wall clock, summed over workgroups), kClProfWords
    // tile mode (R through the chunked code pass on one device): null = segment mode
    const uint32_t* rt_base;      // [nb1 + 1]: R's pass-1 tiles of each cluster
    const uint32_t* rt_start;     // tile -> first pool slot
    const uint32_t* rt_cnt;       // tile -> codes
    const int64_t* r_pool;        // R's chunk pool (codes)
    const uint32_t* err_r;        // R's pass-1 error word (fold_pass1_error), or null
    // k_cluster_probe_big: null, or the host's pinned {count, failed} that the
    // launch's last workgroup writes (no read-back copy after the join); done
    // counts its finished workgroups (zero between launches)
    unsigned long long* host_out;
    uint32_t* done;
    // with host_out: the probe side's chunk state (s_clear16 16-B words),
    // cleared by the last workgroup when the join did not fail (the next
    // join's pass 1 then skips its memset)
    uint4* s_clear;
    uint32_t s_clear16;
};

// A cluster's table is in HBM (k_cluster_big_fill / k_cluster_probe_big):
// more codes than the LDS table holds, or (tile mode) more runs than a build
// reads at once. The three kernels decide it the same way.
__device__ __forceinline__ bool cl_big(uint32_t m, uint32_t runs, uint32_t lim) { return m > lim || runs > kHtSegs; }
// PROF sections of a build: runs + codes of a cluster not prefetched; table
// cleared + the next cluster's runs; inserts; the next cluster's codes requested;
// then the number of builds and of builds not prefetched
constexpr int kClProfWords = 6;

// Cluster d's runs over the segments: sseg[g] = codes before segment g (sseg[nseg] = m),
// sptr[g] = where element r of segment g's run sits, minus r; returns B_d (first code
// over all segments). Wave 0 computes, every thread sees it after the caller's barrier.
// TM: 1 = tile mode, 0 = segment mode, -1 = decided by a.rt_base (the big
// kernels); the probe is instantiated per mode (one path's registers each).
template <int TM = -1>
__device__ __forceinline__ void cl_runs(const ClusterArgs& a, uint32_t d, uint32_t* sseg, const int64_t** sptr,
                                        uint32_t* sB, uint32_t* sM, uint32_t* sN) {
    const uint32_t tid = threadIdx.x;
    if (TM == 1 || (TM == -1 && a.rt_base)) {   // tile mode: the cluster's R tiles are its runs
        if (tid < 64) {
            const uint32_t t0 = a.rt_base[d], nt = a.rt_base[d + 1] - t0;
            uint32_t lo = 0, len = 0;
            if (tid < nt && nt <= static_cast<uint32_t>(kHtSegs)) {
                lo = a.rt_start[t0 + tid];
                len = a.rt_cnt[t0 + tid];
            }
            uint32_t x = len;
#pragma unroll
            for (int o = 1; o < kHtSegs; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (tid >= static_cast<uint32_t>(o)) x += y;
            }
            if (tid < nt && nt <= static_cast<uint32_t>(kHtSegs)) {
                sseg[tid + 1] = x;
                sptr[tid] = a.r_pool + lo - (x - len);
            }
            if (tid == 0) {
                sseg[0] = 0;
                const uint32_t b0 = a.r_bounds[0][d];
                *sB = b0;
                *sM = a.r_bounds[0][d + 1] - b0;
                *sN = nt;
            }
        }
        return;
    }
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
        if (tid == a.nseg - 1) *sM = x;
        if (tid == 0) *sN = a.nseg;
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
// the others return at once (none at the balanced configurations). Their S
// tiles are probed by k_cluster_probe_big after k_cluster_probe (which skips
// them), so the main probe's loop issues the same global loads on every path.
__global__ __launch_bounds__(256) void k_cluster_big_fill(ClusterArgs a) {
    __shared__ uint32_t sseg[kHtSegs + 1];
    __shared__ const int64_t* sptr[kHtSegs];
    __shared__ uint32_t sB, sM, sN;
    const uint32_t d = blockIdx.x, tid = threadIdx.x;
    cl_runs(a, d, sseg, sptr, &sB, &sM, &sN);
    __syncthreads();
    const uint32_t m = sM;
    if (!cl_big(m, sN, a.lim)) return;   // workgroup-uniform
    const uint64_t e = d == 0 ? a.e1 : 0ull;
    const uint32_t cap = cl_big_cap(m);
    uint64_t* t = a.gtab + 4ull * sB + 2ull * d;
    for (uint32_t sl = tid; sl < cap; sl += 256) t[sl] = e;
    __threadfence();
    __syncthreads();
    if (a.rt_base) {   // tile mode: tile by tile
        for (uint32_t ti = a.rt_base[d]; ti < a.rt_base[d + 1]; ti++) {
            const int64_t* src = a.r_pool + a.rt_start[ti];
            const uint32_t c = a.rt_cnt[ti];
            for (uint32_t r = tid; r < c; r += 256) ht_insert(t, cap / 2 - 1, e, static_cast<uint64_t>(src[r]));
        }
        return;
    }
    for (uint32_t r = tid; r < m; r += 256) {
        const uint32_t g = cl_seg_of(sseg, a.nseg, r);
        ht_insert(t, cap / 2 - 1, e, static_cast<uint64_t>(sptr[g][r]));
    }
}

// Whether cluster d takes the HBM table (cl_big), from its sizes alone (one
// thread; the same decision as cl_runs + cl_big).
__device__ __forceinline__ bool cl_is_big(const ClusterArgs& a, uint32_t d) {
    if (a.rt_base) return cl_big(a.r_bounds[0][d + 1] - a.r_bounds[0][d], a.rt_base[d + 1] - a.rt_base[d], a.lim);
    uint32_t m = 0;
    for (uint32_t g = 0; g < a.nseg; g++) m += a.r_bounds[g][d + 1] - a.r_bounds[g][d];
    return cl_big(m, a.nseg, a.lim);
}

// The S tiles of the big clusters against their HBM tables, their tiles from
// the pass-1 tile list. kProbeBigGrid workgroups: each finds the big clusters
// among its share (clusters blockIdx.x + k * grid, one load round) and probes
// them one by one (none at the balanced configurations). host_out: the last
// workgroup to finish copies the count pair to the host.
constexpr uint32_t kProbeBigGrid = 64;
__global__ __launch_bounds__(256) void k_cluster_probe_big(ClusterArgs a) {
    __shared__ uint32_t sseg[kHtSegs + 1];
    __shared__ const int64_t* sptr[kHtSegs];
    __shared__ uint32_t sB, sM, sN;
    __shared__ uint32_t red[4];
    __shared__ uint32_t list[256], nlist;
    const uint32_t tid = threadIdx.x, G = gridDim.x;
    if (tid == 0) nlist = 0;
    __syncthreads();
    for (uint32_t d = blockIdx.x + tid * G; d < a.nb1; d += 256 * G)
        if (cl_is_big(a, d)) list[atomicAdd(&nlist, 1u)] = d;   // (<= 256: nb1 <= 256 * grid)
    __syncthreads();
    const uint32_t nbig = nlist;
    uint32_t hits = 0;
    for (uint32_t k = 0; k < nbig; k++) {
        const uint32_t d = list[k];
        cl_runs(a, d, sseg, sptr, &sB, &sM, &sN);
        __syncthreads();
        const uint64_t e = d == 0 ? a.e1 : 0ull;
        const uint32_t bmask = cl_big_cap(sM) / 2 - 1;
        const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(a.gtab + 4ull * sB + 2ull * d);
        __syncthreads();   // (sB / sM read before the next cluster's cl_runs)
        for (uint32_t t = a.tile_base[d]; t < a.tile_base[d + 1]; t++) {
            const uint32_t lo = a.tile_start[t], c = a.tile_cnt[t];
            for (uint32_t i = tid; i < c; i += 256) {
                const uint64_t cc = static_cast<uint64_t>(a.s_codes[lo + i]);
                uint32_t b = static_cast<uint32_t>(cc >> kHtBucketShift) & bmask;
                for (;;) {
                    const ulonglong2 w = g2[b];
                    if (w.x == cc || w.y == cc) {
                        hits++;
                        break;
                    }
                    if (w.y == e) break;
                    b = (b + 1) & bmask;
                }
            }
        }
    }
    if (nbig == 0 && !a.host_out) return;   // workgroup-uniform
    __shared__ uint32_t clear_state;
    uint32_t x = hits;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = x;
    __syncthreads();
    if (tid == 0) {
        clear_state = 0;
        const unsigned long long s = static_cast<unsigned long long>(red[0]) + red[1] + red[2] + red[3];
        if (s) atomicAdd(a.count, s);
        if (a.host_out) {
            __threadfence();
            if (atomicAdd(a.done, 1u) == G - 1) {   // every other workgroup's count is in
                __threadfence();
                const unsigned long long c0 = atomicAdd(a.count, 0ull), c1 = atomicAdd(a.count + 1, 0ull);
                a.host_out[0] = c0;   // vector stores to fine-grained host memory; the
                __threadfence_system();   // host polls word 1, so word 0 lands first
                a.host_out[1] = c1;
                __threadfence_system();
                atomicExch(a.done, 0u);
                clear_state = a.s_clear && c1 == 0 ? 1u : 0u;
            }
        }
    }
    __syncthreads();
    if (clear_state)
        for (uint32_t i = tid; i < a.s_clear16; i += 256) a.s_clear[i] = make_uint4(0, 0, 0, 0);
}

// The probe. LDS: the cluster table (cap slots) + a few words. PF: tiles
// whose codes are in flight ahead of the one probed (registers: PF * ITEMS codes).
// PRE: while a cluster's tiles are probed, the NEXT cluster's R codes are
// already loaded into registers (its runs staged in the other LDS run buffer
// during this cluster's build), so a build waits on no memory; only the
// first build of a workgroup, or a cluster its range skips, loads in place.
// Inserts by bucket fill counters (16 bits per bucket, after the table in
// LDS: cap bytes): one 32-bit LDS atomic add per bucket tried and a plain
// store, not 64-bit compare-and-swaps slot by slot (measured: builds 0.082 ->
// 0.055 ms at C2). A duplicate R code then takes a second slot (the count is a
// set test: a probe stops at the first match either way); a bucket's attempts
// are at most the cluster's codes (<= lim < 2^16), so a counter never carries
// into its neighbour.
__host__ __device__ constexpr size_t cluster_lds_bytes(uint32_t cap) { return static_cast<size_t>(cap) * 9; }
// ASMW: the S codes' loads in inline assembly, each step waiting for exactly its
// own tile (the compiler, merging the build and staging paths, waited for
// every load in flight, s_waitcnt vmcnt(0), before every tile's table reads)
#ifndef PHJ_CL_ASM
#define PHJ_CL_ASM 1
#endif
template <int BLOCK, int ITEMS, int PF = 1, bool PRE = true, bool PROF = false, bool TM = false, bool ASMW = PHJ_CL_ASM != 0>
__global__ __launch_bounds__(BLOCK) void k_cluster_probe(ClusterArgs a) {
    constexpr int CPL = kClCapMax * 3 / 4 / BLOCK;   // R codes per lane at the limit
    extern __shared__ __attribute__((aligned(16))) uint64_t tab[];   // [cap] + cap / 4 words of fill counters
    uint32_t* const fill = reinterpret_cast<uint32_t*>(tab + a.cap);
    __shared__ uint32_t sseg_[2][kHtSegs + 1];
    __shared__ const int64_t* sptr_[2][kHtSegs];
    __shared__ uint32_t sB_[2], sM_[2], sN_[2];   // first code, codes, runs of the cluster in each run buffer
    __shared__ uint32_t red[BLOCK / 64];
    constexpr uint32_t MR = 512;                 // tiles of metadata staged in LDS at a time
    __shared__ uint32_t smeta[3][MR];            // {cluster, first slot, codes} of tiles mbase .. mbase + MR - 1
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t total = a.tile_base[a.nb1];
    // workgroup -> a contiguous range of tiles; neighbouring ranges on one XCD
    // (they share the cluster at their boundary: its R run is an L2 hit)
    const uint32_t G = gridDim.x, r8 = (blockIdx.x & 7u) * (G >> 3) + (blockIdx.x >> 3);
    const uint32_t t_lo = static_cast<uint32_t>(static_cast<uint64_t>(total) * r8 / G);
    const uint32_t t_hi = static_cast<uint32_t>(static_cast<uint64_t>(total) * (r8 + 1) / G);
    uint32_t hits = 0;
    const unsigned long long clk0 = wall_clock64();
    unsigned long long clk_b = 0;   // wall clock in table builds (workgroup-uniform sections)
    __shared__ unsigned long long prof[PROF ? kClProfWords : 1];   // thread 0's sums (workgroup-uniform sections)
    if (PROF && tid < kClProfWords) prof[tid] = 0;
    if (t_lo < t_hi) {   // workgroup-uniform
        // PF register buffers of tile codes, used in turn (no register moves:
        // a move of a register a load is still writing waits for that load).
        // The step for tile t probes the codes in its buffer (requested PF
        // steps earlier; tiles t + 1 .. t + PF - 1 stay in flight), then
        // requests tile t + PF's codes into the buffer. Every global load of a step
        // is issued on every path, in the same order (indices clamped; a tile
        // past the range reads the last one's chunk with no valid lanes), so a
        // wait covers only what was issued before the awaited load: vmcnt
        // retires in issue order, and one conditional load made the compiler
        // wait for everything in flight. The metadata loads are vector loads (a
        // scalar load would be waited for by every LDS access: lgkmcnt counts both).
        typedef long long v2i __attribute__((ext_vector_type(2)));
        // the tiles' codes, two per 16-B load (kv[f][i / 2] holds items i, i + 1)
        v2i kv[PF][ITEMS / 2];
        uint32_t vm[PF], dq[PF];
        // tile metadata staged in LDS, MR tiles at a time (refilled behind a
        // barrier every MR tiles): the loop's only global loads are then the
        // tiles' codes and the builds' R codes, and an LDS read of metadata
        // never waits for a global load
        uint32_t mbase = 0xffffffffu;
        auto stage = [&](uint32_t base) {   // workgroup-uniform
            __syncthreads();
            for (uint32_t i = tid; i < MR; i += BLOCK) {
                const uint32_t ti = min(base + i, t_hi - 1);
                smeta[0][i] = a.tile_seg[ti];
                smeta[1][i] = a.tile_start[ti];
                smeta[2][i] = a.tile_cnt[ti];
            }
            __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0): this path's loads done (see build)
            __syncthreads();
            mbase = base;
        };
        auto load = [&](uint32_t t, v2i* k, uint32_t& m, uint32_t& dd) {
            if (t - mbase >= MR && t < t_hi) stage(t);   // workgroup-uniform
            const uint32_t j = min(t, t_hi - 1) - mbase;
            dd = smeta[0][j];
            const uint32_t lo = smeta[1][j];
            const uint32_t c = t < t_hi ? smeta[2][j] : 0u;
            m = 0;
            // 16-B loads, two codes per lane each: a tile is one pass-1 chunk of
            // BLOCK * ITEMS allocated slots; element (i, h) = code 2 * (i / 2 *
            // BLOCK + tid) + h. Every lane loads (the same loads on every path),
            // lanes past the tile's codes at its last pair, which they share
            // with a valid lane (masked off: a chain's last, partial chunk is
            // not read whole; ~15 % of the bytes at C2)
            const v2i* src = reinterpret_cast<const v2i*>(a.s_codes + lo);
            const uint32_t last = c ? (c - 1) / 2 : 0u;
#pragma unroll
            for (int i = 0; i < ITEMS; i += 2) {
                const uint32_t e = 2 * ((i / 2) * BLOCK + tid);
                const v2i* ptr = src + min((i / 2) * BLOCK + tid, last);
                if constexpr (ASMW) {
                    // issued outside the compiler's wait model: the step waits for
                    // exactly this tile (CLW below)
                    __asm__ volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(k[i / 2]) : "v"(ptr));
                } else {
                    k[i / 2] = __builtin_nontemporal_load(ptr);
                }
                m |= (e < c ? (1u << i) : 0u) | (e + 1 < c ? (2u << i) : 0u);
            }
        };
        stage(t_lo);
#pragma unroll
        for (int f = 0; f < PF; f++) load(t_lo + f, kv[f], vm[f], dq[f]);   // tiles t_lo .. t_lo + PF - 1
        uint32_t cur = 0xffffffffu, bmask = 0;
        bool big = false;
        uint64_t e = 0;
        uint32_t pb = 0;                 // run buffer of the current cluster
        uint32_t pre = 0xffffffffu;      // the cluster whose codes are in rn[] (PRE)
        uint64_t rn[PRE ? CPL : 1];
        const uint32_t d_last = a.tile_seg[t_hi - 1];   // the range's last cluster
        // codes of the cluster whose runs are in buffer `buf` (m of them), requested at once
        auto fetch = [&](uint32_t buf, uint32_t m, uint64_t* rc) {
            const uint32_t* sseg = sseg_[buf];
            const int64_t* const* sptr = sptr_[buf];
            const uint32_t nrun = TM ? sN_[buf] : a.nseg;   // <= kHtSegs (else the cluster is big)
            // tile mode: m is R's pass-1 cluster size; the runs' sum is smaller
            // only when k_tile_chunks voided a tile (a stale table: the count
            // is failed by err_r), and no read goes past the runs then
            if (TM) m = min(m, sseg[nrun]);
            if (nrun == 1) {   // one run: element r at sptr[0] + r
                const int64_t* src = sptr[0];
#pragma unroll
                for (int j = 0; j < CPL; j++) {
                    const uint32_t r = j * BLOCK + tid;
                    rc[j] = r < m ? static_cast<uint64_t>(src[r]) : 0ull;
                }
            } else {   // the segments' run ends in registers (broadcast reads), searched per element
                uint32_t se[kHtSegs];
#pragma unroll
                for (int g = 0; g < kHtSegs; g++)   // workgroup-uniform: scalar registers
                    se[g] = __builtin_amdgcn_readfirstlane(g < static_cast<int>(nrun) ? sseg[g + 1] : 0xffffffffu);
#pragma unroll
                for (int j = 0; j < CPL; j++) {
                    const uint32_t r = j * BLOCK + tid;
                    uint32_t g = 0;
#pragma unroll
                    for (int q = 0; q < kHtSegs; q++) g += r >= se[q] ? 1u : 0u;   // segments ending at or before r
                    rc[j] = r < m ? static_cast<uint64_t>(sptr[min(g, nrun - 1)][r]) : 0ull;
                }
            }
        };
        // cluster d's table, in LDS (or the descriptor of its HBM table)
        auto build = [&](uint32_t d) {
            __syncthreads();   // every probe of the previous table is done
            const unsigned long long cb = wall_clock64();
            uint64_t rc[CPL];
            if (PROF && tid == 0) prof[PROF ? 5 : 0] += PRE && pre == d ? 0u : 1u;
            if (PRE && pre == d) {   // runs staged in the other buffer, codes in registers
                pb ^= 1u;
#pragma unroll
                for (int j = 0; j < CPL; j++) rc[j] = rn[PRE ? j : 0];
            } else {
                cl_runs<TM ? 1 : 0>(a, d, sseg_[pb], sptr_[pb], &sB_[pb], &sM_[pb], &sN_[pb]);
                __syncthreads();
                const uint32_t m0 = sM_[pb];
                if (!cl_big(m0, sN_[pb], a.lim)) fetch(pb, m0, rc);
                if (PROF) __builtin_amdgcn_s_waitcnt(0xF70);
            }
            unsigned long long c1 = 0, c2 = 0, c3 = 0;
            if (PROF) c1 = wall_clock64();
            const uint32_t m = sM_[pb];
            e = d == 0 ? a.e1 : 0ull;
            big = cl_big(m, sN_[pb], a.lim);
            if (!big) {
                bmask = a.cap / 2 - 1;
                ulonglong2* t2 = reinterpret_cast<ulonglong2*>(tab);
                for (uint32_t b = tid; b <= bmask; b += BLOCK) t2[b] = make_ulonglong2(e, e);
                for (uint32_t w = tid; w < a.cap / 4; w += BLOCK) fill[w] = 0;
            } else {
                bmask = cl_big_cap(m) / 2 - 1;
            }
            // the next cluster's runs into the other buffer (read after the barrier)
            const bool nxt = PRE && d < d_last;
            if (nxt) cl_runs<TM ? 1 : 0>(a, d + 1, sseg_[pb ^ 1u], sptr_[pb ^ 1u], &sB_[pb ^ 1u], &sM_[pb ^ 1u], &sN_[pb ^ 1u]);
            __syncthreads();   // cleared; the next runs staged
            if (PROF) c2 = wall_clock64();
            if (!big) {
                // the home bucket's attempt, then (home full) the walk; the code
                // stored once, after it (a store inside the retry loop, as before,
                // measured build 0.068 -> 0.057 ms at C2, 0.081 -> 0.069 at W = 8:
                // profiles/r06m_*; two or four home attempts in flight per lane
                // were no faster)
#pragma unroll
                for (int j = 0; j < CPL; j++) {
                    if (j * BLOCK + tid < m) {
                        const uint64_t c = rc[j];
                        uint32_t b = static_cast<uint32_t>(c >> kHtBucketShift) & bmask;
                        uint32_t sh = (b & 1u) * 16u;
                        uint32_t p = (atomicAdd(&fill[b >> 1], 1u << sh) >> sh) & 0xffffu;
                        while (p >= 2) {
                            b = (b + 1) & bmask;
                            sh = (b & 1u) * 16u;
                            p = (atomicAdd(&fill[b >> 1], 1u << sh) >> sh) & 0xffffu;
                        }
                        tab[2 * b + p] = c;
                    }
                }
            }
            // every load of the build path complete (s_waitcnt vmcnt(0)): else
            // the compiler, merging this path with the no-build one, makes the
            // next step wait for every load in flight on both
            // (leaving it to the compiler measured the same: r06c_ab_nodrain.txt)
            __builtin_amdgcn_s_waitcnt(0xF70);
            if (PROF) {
                __syncthreads();
                c3 = wall_clock64();
            }
            pre = 0xffffffffu;
            if constexpr (PRE) {   // the next cluster's codes: in flight during this cluster's tiles
                if (nxt) {
                    const uint32_t mn = sM_[pb ^ 1u];
                    if (!cl_big(mn, sN_[pb ^ 1u], a.lim)) {
                        fetch(pb ^ 1u, mn, rn);
                        pre = d + 1;
                    }
                }
            }
            __syncthreads();   // built
            cur = d;
            const unsigned long long c4 = wall_clock64();
            clk_b += c4 - cb;
            if (PROF && tid == 0) {
                prof[0] += c1 - cb;
                prof[PROF ? 1 : 0] += c2 - c1;
                prof[PROF ? 2 : 0] += c3 - c2;
                prof[PROF ? 3 : 0] += c4 - c3;
                prof[PROF ? 4 : 0] += 1;
            }
        };
        const ulonglong2* tb = reinterpret_cast<const ulonglong2*>(tab);
        uint32_t t = t_lo;
        // one tile: take its codes out of buffer f, refill the buffer, probe
        auto step = [&](int f) -> bool {
            const uint32_t cvm = vm[f], d = dq[f];
            if (d != cur) build(d);   // workgroup-uniform
            if constexpr (ASMW) {
                // this tile's loads: every step issues ITEMS / 2 loads, so at most
                // (PF - 1) * ITEMS / 2 issued after them may stay in flight (any
                // other load issued since only makes the wait longer, never short)
                static_assert(ITEMS == 4, "two 16-B loads per tile");
                __asm__ volatile("s_waitcnt vmcnt(%2)" : "+v"(kv[f][0]), "+v"(kv[f][1]) : "n"((PF - 1) * ITEMS / 2));
            }
            int64_t key[ITEMS];
#pragma unroll
            for (int i = 0; i < ITEMS; i += 2) {
                key[i] = kv[f][i / 2].x;
                key[i + 1] = kv[f][i / 2].y;
            }
            if (!big) {   // LDS: every item's home bucket read, then the walks
                ulonglong2 v[ITEMS];
#pragma unroll
                for (int i = 0; i < ITEMS; i++) v[i] = tb[static_cast<uint32_t>(static_cast<uint64_t>(key[i]) >> kHtBucketShift) & bmask];
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    const uint64_t cc = static_cast<uint64_t>(key[i]);
                    bool hit = v[i].x == cc || v[i].y == cc;
                    if ((cvm >> i) & 1u) {
                        if (!hit && v[i].y != e) {
                            uint32_t b = static_cast<uint32_t>(cc >> kHtBucketShift) & bmask;
                            for (;;) {
                                b = (b + 1) & bmask;
                                const ulonglong2 w = tb[b];
                                hit = w.x == cc || w.y == cc;
                                if (hit || w.y == e) break;
                            }
                        }
                        hits += hit ? 1u : 0u;
                    }
                }
            }   // (a big cluster's tiles: k_cluster_probe_big, no global load here)
            // the buffer refilled only now, once its codes are consumed (a refill
            // into other registers would put a move at the loop's back edge,
            // which waits for the refill): tile t + PF's codes; tiles t + 1 ..
            // t + PF - 1 were in flight during this tile's probe
            load(t + PF, kv[f], vm[f], dq[f]);
            return ++t < t_hi;
        };
        bool more = true;
        while (more) {
#pragma unroll
            for (int f = 0; f < PF; f++) {
                more = step(f);
                if (!more) break;
            }
        }
        if constexpr (ASMW) {   // the loads past the range land before their registers are reused
#pragma unroll
            for (int f = 0; f < PF; f++) __asm__ volatile("s_waitcnt vmcnt(0)" : "+v"(kv[f][0]), "+v"(kv[f][1]));
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
        if (a.split) {
            const unsigned long long all = wall_clock64() - clk0;
            atomicAdd(&a.split[0], clk_b);
            atomicAdd(&a.split[1], all - clk_b);
        }
        if (PROF && a.prof)
            for (int w = 0; w < kClProfWords; w++) atomicAdd(&a.prof[w], prof[PROF ? w : 0]);
    }
    fold_pass1_error(a.err, a.count);
    fold_pass1_error(a.err_r, a.count);
}

}  // namespace phj
