// phj_mat.h — join materialisation for gfx950.
//
// The reference's Run() returns an empty Table<JoinedTuple>
// (src/NoPartitioning/HashJoin.hpp:186, RadixCluster/HashJoin.hpp:240) and
// only logs the count; its per-probe result is HashTable::Get(id), the FIRST
// build tuple found for the key (LinearProbing.hpp:160-180), or null. The
// materialised join is therefore one JoinedTuple {id, payloadA, payloadB}
// (src/Common/Table.hpp:27-33) per probe tuple that has a match, with
// payloadA the payload of that one build tuple and payloadB the probe's.
//
// Two steps, both plain streaming work:
//   1. mark: the join writes, per probe tuple (in the order the probe side is
//      stored), the index of its matching build payload or kNoMatch;
//   2. compact: a count per 4096-tuple block, an exclusive scan, and a write
//      kernel that emits the rows of each block in probe order (wave ballots
//      for the positions inside the block).
// Rows come out in the probe side's storage order: input order for
// NoPartitioning, partition order for the radix join (the reference's
// Join() also visits the probe side partition by partition).
#pragma once

#include "phj_join.h"

namespace phj {

constexpr uint32_t kNoMatch = 0xffffffffu;
constexpr uint32_t kMatBlockItems = 16;                       // per thread
constexpr uint32_t kMatBlock = kBlock * kMatBlockItems;       // 4096 probe tuples per compaction block

struct JoinedRow {   // == phj_joined == Common::JoinedTuple
    int64_t id, payload_a, payload_b;
};

// NoPartitioning lookup returning the slot index (b * 7 + slot) of the first
// equal key, walking buckets as np_lookup does.
__device__ __forceinline__ uint32_t np_lookup_slot(const NPBucket* tab, uint32_t nb, uint32_t b, int64_t key) {
    for (uint32_t step = 0; step < nb; step++) {
        const NPBucket& q = tab[b];
        const uint32_t fill = q.fill;
        const uint32_t c = fill < kNPSlots ? fill : kNPSlots;
        for (uint32_t s = 0; s < c; s++)
            if (q.key[s] == key) return b * kNPSlots + s;
        if (fill < kNPSlots) return kNoMatch;
        b = (b + 1 == nb) ? 0 : b + 1;
    }
    return kNoMatch;
}

// NoPartitioning probe with marks: match[i] = payload slot of S[i]'s key.
template <int HK>
__global__ __launch_bounds__(kBlock) void k_np_probe_mark(const longlong2* S, uint64_t nS, const NPBucket* tab,
                                                          NPHome g, uint64_t seed, uint32_t* match,
                                                          unsigned long long* count) {
    __shared__ uint32_t red[kWaves];
    constexpr int IT = 4;   // as k_np_probe: every home bucket of a round requested before any compare
    uint32_t hits = 0;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kBlock * IT;
    for (uint64_t base = static_cast<uint64_t>(blockIdx.x) * kBlock * IT; base < nS; base += stride) {
        int64_t k[IT];
        uint32_t b[IT];
        longlong2 q[IT][4];
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint64_t i = base + static_cast<uint64_t>(j) * kBlock + threadIdx.x;
            k[j] = i < nS ? __builtin_nontemporal_load(&S[i].x) : 0;
        }
#pragma unroll
        for (int j = 0; j < IT; j++) {
            b[j] = np_home_r(hash64<HK>(static_cast<uint64_t>(k[j]), seed), g);
            const longlong2* bp = reinterpret_cast<const longlong2*>(tab + b[j]);
#pragma unroll
            for (int w = 0; w < 4; w++) q[j][w] = bp[w];
        }
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint64_t i = base + static_cast<uint64_t>(j) * kBlock + threadIdx.x;
            if (i >= nS) continue;
            const int64_t key = k[j];
            const uint32_t fill = static_cast<uint32_t>(q[j][3].y);
            const uint32_t c = fill < kNPSlots ? fill : kNPSlots;
            const int64_t ks[kNPSlots] = {q[j][0].x, q[j][0].y, q[j][1].x, q[j][1].y, q[j][2].x, q[j][2].y, q[j][3].x};
            uint32_t m = kNoMatch;
#pragma unroll
            for (int s = kNPSlots - 1; s >= 0; s--)   // the first equal slot wins
                if (static_cast<uint32_t>(s) < c && ks[s] == key) m = b[j] * kNPSlots + s;
            if (m == kNoMatch && fill >= kNPSlots)   // full home bucket: walk on (rare)
                m = np_lookup_slot(tab, g.nb, b[j] + 1 == g.nb ? 0 : b[j] + 1, key);
            match[i] = m;
            hits += m != kNoMatch;
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

// Radix join with marks: the fused per-partition LDS join (k_join_fused's
// structure, one build segment) keeping each LDS key's row in the
// partitioned build relation; match[s] = that row for the partitioned probe
// tuple s. Partitions beyond 256 build keys are joined in rounds; a probe key
// matched in an earlier round keeps its first match.
template <int HK>
__global__ __launch_bounds__(kBlock) void k_join_fused_mark(FusedArgs a, uint32_t* match) {
    constexpr int TCAP = 256, RPL = TCAP / 64, OCAP = TCAP / 2 + 1, KPL = 4;
    constexpr uint32_t SUB = 64 * KPL;
    __shared__ int64_t lk_all[kWaves][TCAP];
    __shared__ uint32_t lr_all[kWaves][TCAP];
    __shared__ uint32_t lo_all[kWaves][OCAP];
    __shared__ uint32_t cur_all[kWaves][OCAP];
    __shared__ unsigned long long red[kWaves];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int64_t* lk = lk_all[wave];
    uint32_t* lr = lr_all[wave];
    uint32_t* loffs = lo_all[wave];
    uint32_t* lcur = cur_all[wave];
    const int64_t* rkeys = a.L.seg[0].keys;
    const uint32_t* rb = a.L.seg[0].bounds;
    unsigned long long hits = 0;
    for (uint32_t item = blockIdx.x * kWaves + wave; item < a.nitems; item += gridDim.x * kWaves) {
        const FusedItem it = a.items[item];
        if (it.s_cnt == 0) continue;
        const uint32_t rlo = rb[it.p], m = rb[it.p + 1] - rlo;
        if (m == 0) continue;
        const uint32_t nsub = (it.s_cnt + SUB - 1) / SUB;
        uint64_t hitbits = 0;   // bit (sub * KPL + j): kFusedChunk / SUB * KPL = 64 bits
        for (uint32_t r0 = 0; r0 < m; r0 += TCAP) {
            const uint32_t mr = min(static_cast<uint32_t>(TCAP), m - r0);
            const uint32_t nbk = table_buckets(mr);
            int64_t rk[RPL];
            uint32_t bk[RPL];
#pragma unroll
            for (int j = 0; j < RPL; j++) {
                const uint32_t f = j * 64 + lane;
                rk[j] = f < mr ? rkeys[rlo + r0 + f] : 0;
            }
            for (uint32_t i = lane; i < nbk; i += 64) lcur[i] = 0;
            wave_lds_sync();
#pragma unroll
            for (int j = 0; j < RPL; j++) {
                bk[j] = bucket_of(hash64<HK>(static_cast<uint64_t>(rk[j]), a.seed), nbk);
                if (static_cast<uint32_t>(j * 64) + lane < mr) atomicAdd(&lcur[bk[j]], 1u);
            }
            wave_lds_sync();
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
                const uint32_t f = j * 64 + lane;
                if (f < mr) {
                    const uint32_t pos = atomicAdd(&lcur[bk[j]], 1u);
                    lk[pos] = rk[j];
                    lr[pos] = rlo + r0 + f;
                }
            }
            wave_lds_sync();
            for (uint32_t sub = 0; sub < nsub; sub++) {
#pragma unroll
                for (int j = 0; j < KPL; j++) {
                    const uint32_t off = sub * SUB + j * 64 + lane;
                    const uint64_t bit = 1ull << (sub * KPL + j);
                    if (off < it.s_cnt && !(hitbits & bit)) {
                        const int64_t key = a.skeys[it.s_lo + off];
                        const uint32_t b = bucket_of(hash64<HK>(static_cast<uint64_t>(key), a.seed), nbk);
                        for (uint32_t t = loffs[b]; t < loffs[b + 1]; t++) {
                            if (lk[t] == key) {
                                match[it.s_lo + off] = lr[t];
                                hitbits |= bit;
                                break;
                            }
                        }
                    }
                }
            }
            wave_lds_sync();   // this round's LDS reads before the next round's stores
        }
        hits += __popcll(hitbits);
    }
    unsigned long long x = hits;
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

// Matches per compaction block -> cnt[block] (cnt has nblocks + 1 entries; the
// exclusive scan turns it into row offsets and the total).
__global__ __launch_bounds__(kBlock) void k_mat_count(const uint32_t* match, uint64_t n, uint32_t* cnt) {
    __shared__ uint32_t red[kWaves];
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kMatBlock;
    uint32_t c = 0;
#pragma unroll
    for (uint32_t j = 0; j < kMatBlockItems; j++) {
        const uint64_t i = base + j * kBlock + threadIdx.x;
        c += (i < n && match[i] != kNoMatch) ? 1u : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kWaves; w++) t += red[w];
        cnt[blockIdx.x] = t;
    }
}

// Rows of one compaction block, in probe order, from offs[block] on. The probe
// side is AoS tuples (sk == nullptr: s_aos) or SoA columns (sk, sp); the build
// payload of a match is rpay[match].
__global__ __launch_bounds__(kBlock) void k_mat_write(const uint32_t* match, uint64_t n, const longlong2* s_aos,
                                                      const int64_t* sk, const int64_t* sp, const int64_t* rpay,
                                                      const uint32_t* offs, JoinedRow* out) {
    __shared__ uint32_t wcnt[kWaves];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kMatBlock;
    uint32_t row = offs[blockIdx.x];
    for (uint32_t j = 0; j < kMatBlockItems; j++) {
        const uint64_t i = base + j * kBlock + threadIdx.x;
        const uint32_t m = i < n ? match[i] : kNoMatch;
        const bool hit = m != kNoMatch;
        const uint64_t bal = __ballot(hit);
        const uint32_t before = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wcnt[wave] = __popcll(bal);
        __syncthreads();
        uint32_t wbase = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) {
            const uint32_t v = wcnt[w];
            wbase += static_cast<uint32_t>(w) < wave ? v : 0u;
            total += v;
        }
        if (hit) {
            int64_t id, pb;
            if (sk) {
                id = sk[i];
                pb = sp[i];
            } else {
                const longlong2 t = s_aos[i];
                id = t.x;
                pb = t.y;
            }
            JoinedRow r;
            r.id = id;
            r.payload_a = rpay[m];
            r.payload_b = pb;
            out[row + wbase + before] = r;
        }
        row += total;
        __syncthreads();   // wcnt reused by the next round
    }
}

}  // namespace phj
