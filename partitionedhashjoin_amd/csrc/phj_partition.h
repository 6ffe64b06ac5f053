// phj_partition.h — radix partition pass kernels for gfx950.
//
// One pass = histogram -> flat exclusive scan -> scatter, per tile of
// T = 256 * ITEMS tuples. This restates, for the GPU, the reference's
// Partition() pipeline (src/RadixCluster/HashJoin.hpp:333-440): scanTable
// (per-worker histogram, :343-357), createPrefixSumTable (exclusive scan
// across workers, :360-390) and partitionTable (stable scatter, :394-412),
// with "worker" = tile. The output is a STABLE partition: partition-major,
// then tile order, then input order inside the tile — the reference's layout.
//
// Segmented passes (pass 2 of a 2-pass radix) partition every pass-1
// partition ("segment") independently: tiles never straddle a segment, and
// the histogram is laid out [segment][digit][tile-in-segment] so one flat
// exclusive scan yields every tile's output offset per digit directly.
//
// Memory shape: input tuples are read once per kernel with 16-B (AoS) or 8-B
// (SoA) per-lane coalesced loads; the scatter sorts the tile locally in LDS
// (wave-level match ranking, stable) and then writes key and payload
// columns with consecutive lanes on consecutive output slots of a digit run.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "phj_hash.h"

namespace phj {

constexpr int kBlock = 256;   // 4 waves of 64
constexpr int kWaves = kBlock / 64;
constexpr int kMaxDigitBits = 11;
constexpr int kMaxBins = 1 << kMaxDigitBits;

// q(key) -> this pass's digit. mode 0: q = h & (P - 1); mode 1: q = h % P
// (Barrett: magic = floor((2^64 - 1) / P), one correction step).
// With sub_bits > 0 (phj_join on large partitions, phj_capi.hip refine_plan)
// q is refined to (q << sub_bits) | sub_bits hash bits taken at sub_shift:
// every partition q stays contiguous and is split into 2^sub_bits
// sub-partitions; equal keys have equal hashes, so they still meet.
struct DigitFn {
    uint64_t seed;
    uint64_t P;
    uint64_t magic;
    uint32_t mode;
    uint32_t shift;
    uint32_t dmask;
    uint32_t sub_bits;
    uint32_t sub_shift;
    uint32_t pad;
};

__host__ __device__ __forceinline__ uint64_t q_from_hash(uint64_t h, const DigitFn& f) {
    uint64_t q;
    if (f.mode == 0) {
        q = h & (f.P - 1);
    } else {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint64_t qt = __umul64hi(h, f.magic);
#else
        const uint64_t qt = static_cast<uint64_t>((static_cast<unsigned __int128>(h) * f.magic) >> 64);
#endif
        q = h - qt * f.P;
        if (q >= f.P) q -= f.P;
    }
    if (f.sub_bits) q = (q << f.sub_bits) | ((h >> f.sub_shift) & ((1ull << f.sub_bits) - 1));
    return q;
}

template <int HK>
__device__ __forceinline__ uint64_t partition_q(uint64_t key, const DigitFn& f) {
    return q_from_hash(hash64<HK>(key, f.seed), f);
}

template <int HK>
__device__ __forceinline__ uint32_t digit_of(uint64_t key, const DigitFn& f) {
    return static_cast<uint32_t>(partition_q<HK>(key, f) >> f.shift) & f.dmask;
}

// Chunked pass 1: up to kShards chains per digit (PassArgs::nshards of them;
// with 8 or 16, shard % 8 is the XCD under round-robin dispatch). The host
// picks about one shard per kTilesPerShard tiles: enough chains that no
// cursor line takes too many atomics, few enough that partial last chunks
// stay a small share of the pass-2 tiles.
constexpr uint32_t kShards = 16;
// A published chunk-table entry (pool chunk ids start at 0). The table is all
// zero between passes: k_tile_chunks clears every entry it reads, so no
// per-pass tag has to reach the kernels (a captured step replays unchanged).
constexpr unsigned long long kPublished = 1ull << 32;
constexpr uint32_t kTilesPerShard = 3072;
__host__ __device__ constexpr size_t chunk_pool_word(uint32_t nb, uint32_t x) { return (static_cast<size_t>(kShards) * nb + 31) / 32 * 32 + 32 * x; }
// the pass's error word: a chunk id or chain index read back out of range
// (a stale chunk table) sets kChunkErr* bits here instead of writing through it
__host__ __device__ constexpr size_t chunk_err_word(uint32_t nb) { return chunk_pool_word(nb, kShards); }
constexpr uint32_t kChunkErrId = 1, kChunkErrIndex = 2, kChunkErrTable = 4;
__host__ __device__ constexpr size_t chunk_hint_word(uint32_t nb) { return chunk_pool_word(nb, 2 * kShards); }
constexpr uint32_t kSinkGroups = 1024;   // k_chunk_codes: workgroups with their own sink words (PassArgs::sink)
__host__ __device__ constexpr size_t chunk_state_bytes(uint32_t nb) { return chunk_hint_word(nb) * 4 + static_cast<size_t>(kShards) * nb * 8; }

struct PassArgs {
    const int64_t* in_keys;     // AoS: tuple base ({id,payload} pairs); SoA: key column
    const int64_t* in_pays;     // SoA payload column (unused for AoS)
    int64_t* out_keys;
    int64_t* out_pays;
    uint32_t* hist;             // [seg][digit][tile]; scanned in place between the kernels
    const uint32_t* seg_bounds; // nseg+1 input offsets; nullptr = one segment [0, n)
    const uint32_t* tile_base;  // nseg+1 cumulative tile counts (segmented passes)
    const uint32_t* tile_seg;   // tile -> segment (segmented passes)
    uint32_t nseg;
    uint32_t n;
    uint32_t ntiles1;           // tiles of the single-segment case
    uint32_t nbins;
    uint32_t nbits;
    uint32_t xcd_remap;         // 1: give each XCD a contiguous run of tiles (grid % 8 == 0)
    uint32_t nt_store;          // 1: scatter stores bypass the caches' allocate (nontemporal)
    uint32_t nt_load;           // 1: tuple loads are nontemporal (keep L2 for the scatter's partial lines)
    uint32_t dig_wide;          // digit column element: 0 = u8, 1 = u16
    void* out_dig;              // pass-1 scatter: writes the NEXT pass's digit per output slot
    const void* in_dig;         // pass-2 histogram: counts this column instead of hashing keys
    uint32_t dig2_mask;         // next pass's digit = q & dig2_mask
    // Chunked pass 1 (no histogram pass): the output is a pool of T-tuple
    // chunks; every digit fills nshards chains of chunks (one per XCD, so the
    // atomic cursors and the chunks' partial lines stay in one L2), so a
    // partition's order is unspecified (not the reference's stable order) but
    // its contents are exact. nullptr = the stable path.
    // chain state (chunk_state_* below): u32 tuples claimed per chain
    // [kShards][nbins], u32 chunks taken from each shard's pool (one 128-B line
    // each), u64 hint per chain = max over its published chunks of
    // ((k + 1) << 32) | id
    uint32_t* chunk_cursor;
    unsigned long long* chunk_tab;  // [kShards][nbins][maxch]: kPublished | pool chunk id of a chain's k-th chunk, 0 = not yet
    const uint32_t* tile_start; // segmented pass over a chunked input: first input slot of each tile ...
    const uint32_t* tile_cnt;   // ... and its tuple count
    uint32_t maxch;             // chunks of one chain (bound)
    uint32_t pool_stride;       // chunks of one shard's pool
    uint32_t nshards;           // chains per digit (<= kShards)
    uint32_t keys_only;         // chunked pass 1 for the counting probe: only the key column is written / read
    unsigned long long* sink;   // k_chunk_codes: [kSinkGroups][BLOCK] words the stores past the tile target (never read)
    DigitFn f;
    unsigned long long* prof;   // k_chunk_codes_pipe PROF: clocks of its phases, kP1ProfWords (diagnostics)
};
constexpr int kP1ProfWords = 16;

// Workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md,
// "Workgroup dispatch"); with xcd_remap each XCD instead walks a contiguous
// run of tiles, so the partial output lines of neighbouring tiles meet in one
// L2. Placement only changes speed, never results.
__device__ __forceinline__ uint32_t tile_id(const PassArgs& a) {
    if (!a.xcd_remap) return blockIdx.x;
    const uint32_t per = gridDim.x >> 3;
    return (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
}

struct TileLoc {
    uint32_t tseg, ntiles_s, tb_s, lo, hi;
};

__device__ __forceinline__ bool locate_tile_rt(const PassArgs& a, uint32_t tile, uint32_t T,
                                               TileLoc& L) {
    if (a.seg_bounds == nullptr) {
        if (tile >= a.ntiles1) return false;
        L.tseg = tile;
        L.ntiles_s = a.ntiles1;
        L.tb_s = 0;
        L.lo = tile * T;
        L.hi = min(a.n, L.lo + T);
        return true;
    }
    const uint32_t total = a.tile_base[a.nseg];
    if (tile >= total) return false;
    const uint32_t l = a.tile_seg[tile];
    L.tb_s = a.tile_base[l];
    L.tseg = tile - L.tb_s;
    L.ntiles_s = a.tile_base[l + 1] - L.tb_s;
    if (a.tile_start) {   // a chunked input: every tile is one chunk of a segment's chains
        L.lo = a.tile_start[tile];
        L.hi = L.lo + a.tile_cnt[tile];
    } else {
        L.lo = a.seg_bounds[l] + L.tseg * T;
        L.hi = min(a.seg_bounds[l + 1], L.lo + T);
    }
    return true;
}

template <int T>
__device__ __forceinline__ bool locate_tile(const PassArgs& a, uint32_t tile, TileLoc& L) {
    return locate_tile_rt(a, tile, T, L);
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = threadIdx.x & 63;
    return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
}

// Lanes of this wave holding the same digit (valid lanes only).
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid, uint32_t nbits) {
    uint64_t m = __ballot(valid);
    for (uint32_t b = 0; b < nbits; b++) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

// Count digit d of this lane (if valid) into the wave's LDS row. Lanes that
// share the first active lane's digit are counted with one add (the common
// case under key skew, where a plain LDS atomic would serialise 64-way).
__device__ __forceinline__ void count_digit(uint32_t* row, uint32_t d, bool valid) {
    const uint64_t act = __ballot(valid);
    if (act == 0) return;
    const uint32_t first = __builtin_amdgcn_readlane(d, __builtin_ctzll(act));
    const uint64_t same = __ballot(valid && d == first);
    const uint32_t lane = threadIdx.x & 63;
    if (valid && d != first) atomicAdd(&row[d], 1u);
    if (lane == static_cast<uint32_t>(__builtin_ctzll(act))) atomicAdd(&row[first], static_cast<uint32_t>(__popcll(same)));
}

// A slot from counter row C for this lane's digit d (every lane calls it,
// d computed on invalid lanes too): the lanes sharing the wave's first active
// digit take one LDS atomic together, so a hot key's digit does not
// serialise a wave-instruction 64-way (Zipf input); the others take one each.
__device__ __forceinline__ uint32_t agg_rank_lds(uint32_t* C, uint32_t d, bool valid) {
    const uint64_t act = __ballot(valid);
    if (act == 0) return 0;
    const int leader = __builtin_ctzll(act);
    const uint32_t ld = __builtin_amdgcn_readlane(d, leader);
    const bool mine = valid && d == ld;
    const uint64_t same = __ballot(mine);
    uint32_t base = 0;
    if ((threadIdx.x & 63) == static_cast<uint32_t>(leader)) base = atomicAdd(&C[ld], static_cast<uint32_t>(__popcll(same)));
    base = __builtin_amdgcn_readlane(base, leader);
    if (mine) return base + static_cast<uint32_t>(__popcll(same & lanemask_lt()));
    return valid ? atomicAdd(&C[d], 1u) : 0u;
}

// Exclusive scan of one value per thread across a block of NW waves.
template <int NW, bool TRAIL = true>
__device__ __forceinline__ uint32_t block_exclusive_scan_t(uint32_t v, uint32_t* tmp,
                                                           uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) tmp[wave] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const uint32_t s = tmp[w];
        if (w < (int)wave) before += s;
        all += s;
    }
    if constexpr (TRAIL) __syncthreads();   // TRAIL = false: the caller's next barriers order tmp's reuse
    total = all;
    return before + x - v;
}

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* tmp,
                                                         uint32_t& total) {
    return block_exclusive_scan_t<kWaves>(v, tmp, total);
}

template <bool AOS>
__device__ __forceinline__ void load_tuple(const PassArgs& a, uint32_t idx, int64_t& k, int64_t& p) {
    if constexpr (AOS) {
        if (a.nt_load) {
            typedef long long v2i __attribute__((ext_vector_type(2)));
            const v2i t = __builtin_nontemporal_load(reinterpret_cast<const v2i*>(a.in_keys) + idx);
            k = t.x;
            p = t.y;
            return;
        }
        const longlong2 t = reinterpret_cast<const longlong2*>(a.in_keys)[idx];
        k = t.x;
        p = t.y;
    } else {
        k = a.in_keys[idx];
        p = a.in_pays[idx];
    }
}

template <bool OUT_AOS>
__device__ __forceinline__ void store_tuple(const PassArgs& a, uint32_t o, int64_t k, int64_t p) {
    if constexpr (OUT_AOS) {
        longlong2* t = reinterpret_cast<longlong2*>(a.out_keys) + o;
        if (a.nt_store) {
            __builtin_nontemporal_store(k, &t->x);
            __builtin_nontemporal_store(p, &t->y);
        } else {
            *t = make_longlong2(k, p);
        }
    } else {
        if (a.nt_store) {
            __builtin_nontemporal_store(k, a.out_keys + o);
            __builtin_nontemporal_store(p, a.out_pays + o);
        } else {
            a.out_keys[o] = k;
            a.out_pays[o] = p;
        }
    }
}

// Pass 1 of a 2-pass partition already hashes every tuple: it leaves the
// pass-2 digit (q & mask, one or two bytes) in a column in output order, so
// the pass-2 histogram reads 1-2 B per tuple instead of the 8-B key (or the
// 16-B tuple).
template <int HK>
__device__ __forceinline__ void store_next_digit(const PassArgs& a, uint32_t o, int64_t key) {
    const uint32_t d2 = static_cast<uint32_t>(partition_q<HK>(static_cast<uint64_t>(key), a.f)) & a.dig2_mask;
    if (a.dig_wide) static_cast<uint16_t*>(a.out_dig)[o] = static_cast<uint16_t>(d2);
    else static_cast<uint8_t*>(a.out_dig)[o] = static_cast<uint8_t>(d2);
}

// Per-tile digit histogram -> hist[(tb_s * nbins) + d * ntiles_s + tseg].
template <int BLOCK, int ITEMS, bool AOS, int HK>
__global__ __launch_bounds__(BLOCK) void k_hist(PassArgs a) {
    __builtin_amdgcn_s_setprio(3);   // (R's chain beside S's persistent pass 1: issue first)
    constexpr int NW = BLOCK / 64;
    constexpr int T = BLOCK * ITEMS;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(smem);  // [NW][nbins]
    TileLoc L;
    if (!locate_tile<T>(a, tile_id(a), L)) return;
    const uint32_t nb = a.nbins;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (uint32_t i = tid; i < NW * nb; i += BLOCK) wcnt[i] = 0;
    uint32_t* my = wcnt + wave * nb;
    // Order does not matter for a histogram, so every lane loads 16 B (one AoS
    // tuple, or two consecutive keys of a SoA key column: aligned pairs) and
    // counts into its wave's private LDS row (count_digit).
    if constexpr (AOS) {
        const uint32_t cnt = L.hi - L.lo;
        int64_t key[ITEMS];
        const uint32_t wbase = wave * 64 * ITEMS;
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = wbase + i * 64 + lane;
            key[i] = e < cnt ? reinterpret_cast<const longlong2*>(a.in_keys)[L.lo + e].x : 0;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = wbase + i * 64 + lane;
            const bool valid = e < cnt;
            count_digit(my, valid ? digit_of<HK>(static_cast<uint64_t>(key[i]), a.f) : 0u, valid);
        }
    } else {
        constexpr int NP = ITEMS / 2 + 1;   // aligned pairs covering [lo, hi)
        const uint32_t plo = L.lo >> 1, phi = (L.hi + 1) >> 1;
        longlong2 kp[NP];
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const uint32_t pi = plo + i * BLOCK + tid;
            kp[i] = pi < phi ? reinterpret_cast<const longlong2*>(a.in_keys)[pi] : make_longlong2(0, 0);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NP; i++) {
            const uint32_t e0 = 2 * (plo + i * BLOCK + tid);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t e = e0 + h;
                const int64_t k = h ? kp[i].y : kp[i].x;
                const bool valid = e >= L.lo && e < L.hi;
                count_digit(my, valid ? digit_of<HK>(static_cast<uint64_t>(k), a.f) : 0u, valid);
            }
        }
    }
    __syncthreads();
    uint32_t* out = a.hist + static_cast<size_t>(L.tb_s) * nb + L.tseg;
    for (uint32_t d = tid; d < nb; d += BLOCK) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) c += wcnt[w * nb + d];
        out[static_cast<size_t>(d) * L.ntiles_s] = c;
    }
}

// Per-tile histogram of a digit column (pass 2 after store_next_digit). A
// tile's digits are only T bytes, so one WAVE counts one tile (16-B loads,
// count_digit into the wave's own LDS row) and writes that tile's column:
// no cross-wave reduction, 1/NW of the counter zeroing.
// tile(wave) = tile_id(block) * 4 + wave; grid covers ceil(tiles / 4) blocks.
template <int T, typename DT>
__global__ __launch_bounds__(256) void k_hist_col(PassArgs a) {
    constexpr int EPC = 16 / static_cast<int>(sizeof(DT));          // digits per 16-B chunk
    constexpr int ROUNDS = (T / EPC + 1 + 63) / 64;                  // chunks covering a tile, per lane
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t nb = a.nbins;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* my = reinterpret_cast<uint32_t*>(smem) + wave * nb;
    TileLoc L;
    if (!locate_tile<T>(a, tile_id(a) * 4 + wave, L)) return;   // wave-uniform; no block barrier below
    for (uint32_t i = lane; i < nb; i += 64) my[i] = 0;
    const uint32_t c0 = L.lo / EPC, c1 = (L.hi + EPC - 1) / EPC;
    const uint4* col = static_cast<const uint4*>(a.in_dig);
    uint4 v[ROUNDS];
#pragma unroll
    for (int r = 0; r < ROUNDS; r++) {
        const uint32_t ci = c0 + r * 64 + lane;
        v[r] = ci < c1 ? col[ci] : make_uint4(0, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
    // each lane walks its 16 consecutive digits and merges runs of equal digits
    // before adding (one LDS add per run: a skewed tile of one hot key costs one
    // add per lane per chunk, a uniform one about one per digit)
#pragma unroll
    for (int r = 0; r < ROUNDS; r++) {
        const uint32_t e0 = (c0 + r * 64 + lane) * EPC;
        const uint32_t w[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
        uint32_t prev = 0, cnt = 0;
#pragma unroll
        for (int j = 0; j < EPC; j++) {
            const uint32_t e = e0 + j;
            const uint32_t d = sizeof(DT) == 1 ? (w[j >> 2] >> (8 * (j & 3))) & 0xffu
                                               : (w[j >> 1] >> (16 * (j & 1))) & 0xffffu;
            if (e >= L.lo && e < L.hi) {
                if (cnt && d == prev) {
                    cnt++;
                } else {
                    if (cnt) atomicAdd(&my[prev], cnt);
                    prev = d;
                    cnt = 1;
                }
            }
        }
        if (cnt) atomicAdd(&my[prev], cnt);
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t* out = a.hist + static_cast<size_t>(L.tb_s) * nb + L.tseg;
    for (uint32_t d = lane; d < nb; d += 64) out[static_cast<size_t>(d) * L.ntiles_s] = my[d];
}

// LDS bytes of k_scatter for a tile of T tuples, nb digits, NW waves.
// The per-tuple digit is kept as one byte when nb <= 256 (two otherwise).
// A chunked pass 1 adds one word per digit. At T = 4096, nb = 256, NW = 8
// that is 80,960 B: still two workgroups per CU.
__host__ __device__ constexpr size_t scatter_lds_bytes(int T, uint32_t nb, int NW = kWaves, bool chunked = false) {
    return static_cast<size_t>(T) * (nb <= 256 ? 17 : 18) + static_cast<size_t>(nb) * 4 * (NW + (chunked ? 3 : 2)) + (chunked ? 128 : 64);
}

// Sorted-digit array of the scatter kernels: u8 for nb <= 256, else u16.
struct SortedDigits {
    void* p;
    bool d8;
    __device__ __forceinline__ void put(uint32_t i, uint32_t d) const {
        if (d8) static_cast<uint8_t*>(p)[i] = static_cast<uint8_t>(d);
        else static_cast<uint16_t*>(p)[i] = static_cast<uint16_t>(d);
    }
    __device__ __forceinline__ uint32_t get(uint32_t i) const {
        return d8 ? static_cast<const uint8_t*>(p)[i] : static_cast<const uint16_t*>(p)[i];
    }
    __device__ __forceinline__ void* end(uint32_t T) const {
        return static_cast<unsigned char*>(p) + (d8 ? T : 2 * T);
    }
};

// Stable scatter of one tile using the scanned offsets.
template <int BLOCK, int ITEMS, bool AOS, bool OUT_AOS, int HK>
__global__ __launch_bounds__(BLOCK) void k_scatter(PassArgs a) {
    constexpr int NW = BLOCK / 64;
    constexpr int T = BLOCK * ITEMS;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t nb = a.nbins;
    int64_t* skey = reinterpret_cast<int64_t*>(smem);
    int64_t* spay = skey + T;
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(spay + T);  // [NW][nb]
    uint32_t* gofs = wcnt + NW * nb;
    uint32_t* dstart = gofs + nb;
    uint32_t* tmp = dstart + nb;                              // 16 words
    const SortedDigits sdig{tmp + 16, nb <= 256};             // [T]

    TileLoc L;
    if (!locate_tile<T>(a, tile_id(a), L)) return;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t cnt = L.hi - L.lo;
    for (uint32_t i = tid; i < NW * nb; i += BLOCK) wcnt[i] = 0;
    {
        const uint32_t* h = a.hist + static_cast<size_t>(L.tb_s) * nb + L.tseg;
        for (uint32_t d = tid; d < nb; d += BLOCK) gofs[d] = h[static_cast<size_t>(d) * L.ntiles_s];
    }
    int64_t key[ITEMS], pay[ITEMS];
    uint32_t dig[ITEMS], rank[ITEMS];
    const uint32_t wbase = wave * 64 * ITEMS;
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const uint32_t e = wbase + i * 64 + lane;
        key[i] = 0;
        pay[i] = 0;
        if (e < cnt) load_tuple<AOS>(a, L.lo + e, key[i], pay[i]);
    }
    __syncthreads();
    // stable ranking: wave-major, then round i, then lane
    uint32_t* my = wcnt + wave * nb;
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const uint32_t e = wbase + i * 64 + lane;
        const bool valid = e < cnt;
        const uint32_t d = valid ? digit_of<HK>(static_cast<uint64_t>(key[i]), a.f) : 0u;
        const uint64_t peers = match_digit(d, valid, a.nbits);
        dig[i] = d;
        rank[i] = 0;
        if (valid) {
            const uint32_t before = my[d];
            const uint64_t lt = peers & lanemask_lt();
            rank[i] = before + __popcll(lt);
            if (lt == 0) my[d] = before + __popcll(peers);
        }
    }
    __syncthreads();
    // digit totals -> tile-local digit starts and per-wave starts
    {
        const uint32_t dpt = (nb + BLOCK - 1) / BLOCK;
        const uint32_t d0 = tid * dpt;
        uint32_t local = 0;
        for (uint32_t j = 0; j < dpt; j++) {
            const uint32_t d = d0 + j;
            if (d < nb) {
#pragma unroll
                for (int w = 0; w < NW; w++) local += wcnt[w * nb + d];
            }
        }
        uint32_t total;
        uint32_t run = block_exclusive_scan_t<NW>(local, tmp, total);
        for (uint32_t j = 0; j < dpt; j++) {
            const uint32_t d = d0 + j;
            if (d < nb) {
                dstart[d] = run;
#pragma unroll
                for (int w = 0; w < NW; w++) {
                    const uint32_t c = wcnt[w * nb + d];
                    wcnt[w * nb + d] = run;
                    run += c;
                }
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const uint32_t e = wbase + i * 64 + lane;
        if (e < cnt) {
            const uint32_t pos = my[dig[i]] + rank[i];
            skey[pos] = key[i];
            spay[pos] = pay[i];
            sdig.put(pos, dig[i]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const uint32_t k = i * BLOCK + tid;
        if (k < cnt) {
            const uint32_t d = sdig.get(k);
            const uint32_t o = gofs[d] + (k - dstart[d]);
            store_tuple<OUT_AOS>(a, o, skey[k], spay[k]);
            if (a.out_dig) store_next_digit<HK>(a, o, skey[k]);
        }
    }
}

// Chunked pass 1 of a 2-pass partition (unordered partitions, PHJ_PART_STABLE
// unset): the same tile sort as k_scatter, but with no histogram pass before
// it. The output is a pool of T-slot chunks; digit d of shard x (the
// workgroup's XCD under round-robin dispatch) fills its own chain of chunks
// through an atomic cursor. So a partition's order is unspecified, its
// contents exact. The relation is read once (16 B/tuple) instead of twice.
//
// Persistent: gridDim = nshards * slots workgroups, shard x walks tiles
// [x * per, (x + 1) * per) with stride `slots`. The cursor round trip of tile
// i is in flight together with the loads of tile i + 1 (issued once tile i
// sits in LDS), so each tile waits on about one memory round trip, as the
// stable scatter does.
//
// Chunk protocol (host guarantees nb <= BLOCK, so digit d = thread d, and
// T-slot chunks, so a run spans at most two): a run that STARTS a chunk
// takes a pool chunk (the tile's two static reservations first) and
// publishes it in the chain's table and hint; it never waits before
// publishing. A run that continues a chunk reads the id from the hint it
// loaded beside its cursor add, or else waits for the table entry: that
// chunk's owner claimed earlier, so it is resident and publishes without
// waiting, and the wait always ends.
//
// VAR bit 0 (the tile's order is free here): rank by one LDS atomic per tuple
// on a single per-digit counter row instead of the stable 64-lane match
// ranking (nbits + 1 ballots per tuple). VAR bit 1: the sorted tile is held as
// 16-B tuples (one ds_write_b128 / ds_read_b128 per tuple instead of two
// 8-B column accesses). The host launches VAR 3; the keys-only hash-code form
// the counting probe consumes is k_chunk_codes below.
template <int BLOCK, int ITEMS, int HK, int VAR = 0>
__global__ __launch_bounds__(BLOCK)
__attribute__((amdgpu_waves_per_eu((BLOCK * ITEMS <= 4096 ? 2 : 1) * BLOCK / 256)))   // what the LDS lets share a CU
void k_scatter_chunked(PassArgs a, uint32_t ntiles, uint32_t per) {
    constexpr int NW = BLOCK / 64;
    constexpr int T = BLOCK * ITEMS;
    constexpr bool ARANK = (VAR & 1) != 0, LAOS = (VAR & 2) != 0;
    // atomic ranking + one 16-B access per element: a digit's three write
    // offsets packed in one 16-B LDS entry (one ds_read_b128 per element in
    // the write loop), placed in the counter rows the atomic ranking leaves unused
    constexpr bool PACK = ARANK && LAOS && NW >= 8;
    constexpr int NWR = ARANK ? 1 : NW;   // counter rows
    // atomic ranking: two counter rows used alternately, so a tile's row is
    // zeroed while the previous one is still read and the loop needs four
    // barriers per tile instead of seven
    constexpr bool DB = ARANK;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t nb = a.nbins;
    int64_t* skey = reinterpret_cast<int64_t*>(smem);
    int64_t* spay = skey + T;
    longlong2* stup = reinterpret_cast<longlong2*>(smem);     // LAOS: [T] tuples over skey/spay
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(spay + T);  // [NW][nb]
    uint32_t* gofs = wcnt + NW * nb;                          // [nb] k <  dsplit: slot = gofs + k
    uint32_t* dstart = gofs + nb;                             // [nb] k >= dsplit: slot = dstart + k
    uint32_t* tmp = dstart + nb;                              // 32 words: [0, NW) scan, 16-17 reservations, 18 bad tile
    const SortedDigits sdig{tmp + 32, nb <= 256};             // [T]
    uint32_t* dsplit = static_cast<uint32_t*>(sdig.end(T));   // [nb]
    uint4* wdesc = reinterpret_cast<uint4*>(wcnt + (((DB ? 2u : 1u) * nb + 3u) & ~3u));   // PACK: [nb] {k < split: slot - k, else, split}

    const uint32_t x = blockIdx.x % a.nshards, slots = gridDim.x / a.nshards;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t t_end = min(ntiles, (x + 1) * per);
    uint32_t tile = x * per + blockIdx.x / a.nshards;
    if (tile >= t_end) return;
    const uint32_t wbase = wave * 64 * ITEMS;
    uint32_t* curs = a.chunk_cursor + static_cast<size_t>(x) * nb;   // this shard's chains
    uint32_t* pool = a.chunk_cursor + chunk_pool_word(nb, x);
    uint32_t* errw = a.chunk_cursor + chunk_err_word(nb);
    const uint32_t id_lo = x * a.pool_stride, id_hi = id_lo + a.pool_stride;   // shard x's pool chunks
    unsigned long long* hints = reinterpret_cast<unsigned long long*>(a.chunk_cursor + chunk_hint_word(nb)) + static_cast<size_t>(x) * nb;
    auto cur = [&](uint32_t d) { return curs + d; };
    auto hint_of = [&](uint32_t d) { return hints + d; };

    // Every wave issues the same memory operations on every path (clamped
    // indices, zero adds) so the compiler's vmcnt bookkeeping stays exact and
    // the waits below cover only what they need, not the prefetch behind them.
    int64_t key[ITEMS], pay[ITEMS];
    const longlong2* rel = reinterpret_cast<const longlong2*>(a.in_keys);
    auto load = [&](uint32_t t) {
        const uint32_t lo = t * T;
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t ix = min(lo + wbase + i * 64 + lane, a.n - 1);
            if (a.nt_load) {
                typedef long long v2i __attribute__((ext_vector_type(2)));
                const v2i v = __builtin_nontemporal_load(reinterpret_cast<const v2i*>(rel) + ix);
                key[i] = v.x;
                pay[i] = v.y;
            } else {
                const longlong2 v = rel[ix];
                key[i] = v.x;
                pay[i] = v.y;
            }
        }
    };
    load(tile);
    uint32_t par = 0;   // DB: this tile's counter row
    if constexpr (DB) {
        for (uint32_t i = tid; i < 2 * nb; i += BLOCK) wcnt[i] = 0;
        __syncthreads();
    }

    for (;;) {
        const uint32_t lo = tile * T, cnt = min(static_cast<uint32_t>(T), a.n - lo);
        if constexpr (!DB) {
            for (uint32_t i = tid; i < NWR * nb; i += BLOCK) wcnt[i] = 0;
            __syncthreads();
        }
        uint32_t dig[ITEMS], rank[ITEMS];
        uint32_t* const crow = wcnt + par * nb;   // DB: this tile's counter row
        uint32_t* my = DB ? crow : wcnt + (ARANK ? 0u : wave * nb);
        const uint32_t next = tile + slots;
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = wbase + i * 64 + lane;
            const bool valid = e < cnt;
            const uint32_t d = valid ? digit_of<HK>(static_cast<uint64_t>(key[i]), a.f) : 0u;
            dig[i] = d;
            rank[i] = 0;
            if constexpr (ARANK) {
                rank[i] = valid ? atomicAdd(&my[d], 1u) : 0u;
            } else {
                const uint64_t peers = match_digit(d, valid, a.nbits);
                if (valid) {
                    const uint32_t before = my[d];
                    const uint64_t lt = peers & lanemask_lt();
                    rank[i] = before + __popcll(lt);
                    if (lt == 0) my[d] = before + __popcll(peers);
                }
            }
        }
        __syncthreads();
        // digit totals (d = tid) -> tile-local starts; claim the run in the chain
        uint32_t c = 0, ds = 0, v0 = 0;
        unsigned long long hint = 0;
        {
            uint32_t* const rows = DB ? crow : wcnt;
            if (tid < nb) {
#pragma unroll
                for (int w = 0; w < NWR; w++) c += rows[w * nb + tid];
            }
            uint32_t total;
            uint32_t run = block_exclusive_scan_t<NW, !DB>(c, tmp, total);
            ds = run;
            if (tid < nb) {
#pragma unroll
                for (int w = 0; w < NWR; w++) {
                    const uint32_t v = rows[w * nb + tid];
                    rows[w * nb + tid] = run;
                    run += v;
                }
            }
            if (tid < nb && c) {
                v0 = atomicAdd(cur(tid), c);
                hint = __hip_atomic_load(hint_of(tid), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (tid == 0) {
                // the tile's reserved pool chunks are static: shard x's pool keeps
                // its first 2 * per chunks for its tiles, two each
                tmp[16] = id_lo + 2 * (tile - x * per);
                tmp[17] = 0;
                tmp[18] = 0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = wbase + i * 64 + lane;
            if (e < cnt) {
                const uint32_t pos = my[dig[i]] + rank[i];
                if constexpr (LAOS) {
                    stup[pos] = make_longlong2(key[i], pay[i]);
                } else {
                    skey[pos] = key[i];
                    spay[pos] = pay[i];
                }
                sdig.put(pos, dig[i]);
            }
        }
        if constexpr (DB) {
            // the next tile's row: its last readers (the previous tile's
            // scatter) are behind this tile's barriers; the barrier below
            // orders these zeros before the next tile's atomics
            uint32_t* const other = wcnt + (par ^ 1u) * nb;
            for (uint32_t i = tid; i < nb; i += BLOCK) other[i] = 0;
        }
        // the tile is in LDS: the next tile's loads go out behind the claims,
        // into the same registers
        load(next < t_end ? next : tile);   // unconditional (a last one goes unused): exact vmcnt waits
        if (tid < nb && c) {
            const uint32_t d = tid;
            const uint32_t off = v0 % T, k0 = v0 / T, k1 = (v0 + c - 1) / T;
            unsigned long long* tab = a.chunk_tab + (static_cast<size_t>(x) * nb + d) * a.maxch;
            auto take = [&]() -> uint32_t {
                const uint32_t r = atomicAdd(&tmp[17], 1u);
                if (r < 2) return tmp[16] + r;
                return id_lo + 2 * per + atomicAdd(pool, 1u);
            };
            auto publish = [&](uint32_t k, uint32_t id) {
                if (k >= a.maxch) return;   // flagged below
                __hip_atomic_store(&tab[k], kPublished | id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicMax(hint_of(d), (static_cast<unsigned long long>(k + 1) << 32) | id);
            };
            uint32_t id0 = id_lo, id1 = id_lo;
            if (off == 0) {
                id0 = take();
                publish(k0, id0);
            }
            if (k1 != k0) {
                id1 = take();
                publish(k1, id1);
            }
            uint32_t bad = k1 >= a.maxch ? kChunkErrIndex : 0u;
            if (off != 0) {
                if ((hint >> 32) == k0 + 1ull) {
                    id0 = static_cast<uint32_t>(hint);
                } else if (k0 < a.maxch) {
                    unsigned long long v;
                    while (((v = __hip_atomic_load(&tab[k0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) == 0)
                        __builtin_amdgcn_s_sleep(2);
                    id0 = static_cast<uint32_t>(v);
                }
            }
            if (id0 < id_lo || id0 >= id_hi || id1 < id_lo || id1 >= id_hi) bad |= kChunkErrId;
            if (bad) {   // a stale chunk table: no store of this tile goes through it
                tmp[18] = 1;
                atomicOr(errw, bad);
            }
            // sorted element k of digit d goes to chain slot v0 + (k - ds)
            const uint32_t split = ds + (T - off);
            if constexpr (PACK) {
                wdesc[d] = make_uint4(id0 * T + off - ds, id1 * T - split, split, 0u);
            } else {
                gofs[d] = id0 * T + off - ds;      // k <  split: chunk k0
                dstart[d] = id1 * T - split;       // k >= split: chunk k1 (uint32 wrap-around)
                dsplit[d] = split;
            }
        }
        __syncthreads();
        const uint32_t lim = tmp[18] ? 0u : cnt;
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t k = i * BLOCK + tid;
            if (k < lim) {
                const uint32_t d = sdig.get(k);
                uint32_t o;
                if constexpr (PACK) {
                    const uint4 w = wdesc[d];
                    o = (k < w.z ? w.x : w.y) + k;
                } else {
                    o = (k < dsplit[d] ? gofs[d] : dstart[d]) + k;
                }
                int64_t tk, tp;
                if constexpr (LAOS) {
                    const longlong2 t = stup[k];
                    tk = t.x;
                    tp = t.y;
                } else {
                    tk = skey[k];
                    tp = spay[k];
                }
                store_tuple<true>(a, o, tk, tp);
                if (a.out_dig) store_next_digit<HK>(a, o, tk);
            }
        }
        if (next >= t_end) break;
        tile = next;
        par ^= 1u;
        // LDS reads of this tile's stores before the next tile's LDS writes:
        // with DB the next tile's first LDS write to skey / wdesc / tmp comes
        // after its ranking barrier
        if constexpr (!DB) __syncthreads();
    }
}

// LDS of k_chunk_codes: the sorted tile, two counter rows, the packed slot
// descriptors and 32 words of scan / reservation state
__host__ __device__ constexpr size_t chunk_codes_lds_bytes(int T, uint32_t nb) {
    return static_cast<size_t>(T) * 8 + (static_cast<size_t>(2 * nb + 3) / 4 * 4 + 4 * static_cast<size_t>(nb)) * 4 + 128;
}

// Chunked pass 1, code form: the S side of the counting on-chip join
// (HashJoin.hpp:295-301 reads only the key, so only the key's hash code goes
// out: 8 B per tuple, phj_hash.h kHashed). Same chunk protocol and output as
// k_scatter_chunked (VAR 3 there), laid out for the memory pipeline:
//  - the next tile's loads go out right after this tile is hashed, so they are
//    in flight through the ranking, the claims and the write-out;
//  - every lane issues the same global operations on every path (see the
//    sink words below): vmcnt retires in issue order and the compiler counts
//    only what every path issues, so one skipped instruction would make the
//    next tile's first wait a wait for this tile's stores as well;
//  - two counter rows used alternately: four barriers per tile, not seven.
// (Deferring the claims' resolution by a tile was measured 0.5 ms slower at
// 200M: a chunk's owner then publishes its id a tile late and the runs that
// continue the chunk wait for it.)
//  - DPT digits per thread (nb <= DPT * BLOCK): thread t owns digits
//    [t * DPT, (t + 1) * DPT) for the scan, the claims and the chain protocol
//    (DPT > 1: the cluster plans of the LDS join, up to 2048 digits).
// Chunk ids and chain indices read back from memory (hint, chunk table) or
// taken from the pool are bound-checked: one out of range (a stale table)
// sets the pass's error word and the tile's stores go to the sink words.
template <int BLOCK, int ITEMS, int HK, int DPT = 1>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(2 * BLOCK / 256)))
void k_chunk_codes(PassArgs a, uint32_t ntiles, uint32_t per) {
    constexpr int NW = BLOCK / 64;
    constexpr int T = BLOCK * ITEMS;
    static_assert(NW <= 16, "scan words [0, NW) below the reservation words");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t nb = a.nbins;   // host: nb <= DPT * BLOCK
    int64_t* sbuf = reinterpret_cast<int64_t*>(smem);                       // [T] sorted codes
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(sbuf + T);                 // [2][nb] counter rows
    uint4* wdesc = reinterpret_cast<uint4*>(wcnt + (2 * nb + 3u) / 4 * 4);  // [nb] {k < split: slot - k, else, split}
    uint32_t* tmp = reinterpret_cast<uint32_t*>(wdesc + nb);                // [0, NW) scan; 16, 17 reservations; 18 bad tile

    const uint32_t x = blockIdx.x % a.nshards, slots = gridDim.x / a.nshards;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t t_end = min(ntiles, (x + 1) * per);
    uint32_t tile = x * per + blockIdx.x / a.nshards;
    if (tile >= t_end) return;
    const uint32_t wbase = wave * 64 * ITEMS;
    uint32_t* curs = a.chunk_cursor + static_cast<size_t>(x) * nb;   // this shard's chains
    uint32_t* pool = a.chunk_cursor + chunk_pool_word(nb, x);
    uint32_t* errw = a.chunk_cursor + chunk_err_word(nb);
    unsigned long long* hints = reinterpret_cast<unsigned long long*>(a.chunk_cursor + chunk_hint_word(nb)) + static_cast<size_t>(x) * nb;
    const uint32_t id_lo = x * a.pool_stride, id_hi = id_lo + a.pool_stride;   // shard x's pool chunks
    // a code's digit; pow2 = the plan's uniform power-of-two form (q = h & (P - 1),
    // no refinement), hoisted out of the per-element loops
    const bool pow2q = a.f.mode == 0 && a.f.sub_bits == 0;
    auto code_digit = [&](uint64_t h, auto pow2) -> uint32_t {
        if constexpr (decltype(pow2)::value) return static_cast<uint32_t>((h & (a.f.P - 1)) >> a.f.shift) & a.f.dmask;
        else return static_cast<uint32_t>(q_from_hash(h, a.f) >> a.f.shift) & a.f.dmask;
    };
    // sink words: a lane without an element stores to its own word here
    // instead of branching round the store
    int64_t* const ssink = reinterpret_cast<int64_t*>(a.sink + static_cast<size_t>(blockIdx.x % kSinkGroups) * BLOCK + tid);

    int64_t key[ITEMS];
    const longlong2* rel = reinterpret_cast<const longlong2*>(a.in_keys);
    auto load = [&](uint32_t t) {   // clamped: the same loads on every path
        const uint32_t lo = t * T;
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t ix = min(lo + wbase + i * 64 + lane, a.n - 1);
            if (a.nt_load) key[i] = __builtin_nontemporal_load(&rel[ix].x);
            else key[i] = rel[ix].x;
        }
    };

    for (uint32_t i = tid; i < 2 * nb; i += BLOCK) wcnt[i] = 0;
    load(tile);
    // the loop's entry mirrors its back edge (loads, then ITEMS stores), so the
    // first waits need not assume an empty queue
    {
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            __hip_atomic_store(ssink, 0ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __asm__ volatile("" ::: "memory");
        }
    }
    __syncthreads();
    uint32_t par = 0;   // this tile's counter row
    for (;;) {
        const uint32_t cnt = min(static_cast<uint32_t>(T), a.n - tile * T);
        const uint32_t next = tile + slots;
        uint32_t* const crow = wcnt + par * nb;
        int64_t code[ITEMS];
        uint32_t dig[ITEMS], rank[ITEMS];
        auto hash_all = [&](auto pow2) {
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                const uint64_t h = hash64<HK>(static_cast<uint64_t>(key[i]), a.f.seed);
                code[i] = static_cast<int64_t>(h);
                dig[i] = wbase + i * 64 + lane < cnt ? code_digit(h, pow2) : 0u;
            }
        };
        if (pow2q) hash_all(std::true_type{});
        else hash_all(std::false_type{});
        load(next < t_end ? next : tile);   // unconditional (a last one goes unused)
        // one LDS atomic per code, back to back (an invalid lane adds 0 to
        // digit 0; measured: plain atomics beat the wave-aggregated
        // agg_rank_lds here by 0.15 ms at 200M)
#pragma unroll
        for (int i = 0; i < ITEMS; i++) rank[i] = atomicAdd(&crow[dig[i]], wbase + i * 64 + lane < cnt ? 1u : 0u);
        __syncthreads();
        // digit totals (thread tid: digits d0 .. d0 + DPT - 1) -> tile-local
        // starts; claim the runs in the chains
        const uint32_t d0 = tid * DPT;
        uint32_t c[DPT], ds[DPT], v0[DPT];
        unsigned long long hint[DPT];
        uint32_t local = 0;
#pragma unroll
        for (int j = 0; j < DPT; j++) {
            c[j] = d0 + j < nb ? crow[d0 + j] : 0u;
            local += c[j];
        }
        uint32_t total;
        uint32_t run = block_exclusive_scan_t<NW, false>(local, tmp, total);
#pragma unroll
        for (int j = 0; j < DPT; j++) {
            ds[j] = run;
            if (d0 + j < nb) crow[d0 + j] = run;
            run += c[j];
            v0[j] = 0;
            hint[j] = 0;
        }
#pragma unroll
        for (int j = 0; j < DPT; j++) {
            if (c[j]) {   // waited for below, in this tile: a conditional issue costs no wait
                v0[j] = atomicAdd(curs + d0 + j, c[j]);
                hint[j] = __hip_atomic_load(hints + d0 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (tid == 0) {
            // the tile's reserved pool chunks are static: shard x's pool keeps
            // its first 2 * per chunks for its tiles, two each
            tmp[16] = id_lo + 2 * (tile - x * per);
            tmp[17] = 0;
            tmp[18] = 0;
        }
        __syncthreads();
        {
            uint32_t base[ITEMS];
#pragma unroll
            for (int i = 0; i < ITEMS; i++) base[i] = crow[dig[i]];
#pragma unroll
            for (int i = 0; i < ITEMS; i++)
                if (wbase + i * 64 + lane < cnt) sbuf[base[i] + rank[i]] = code[i];
            // the next tile's counter row (its last reader, the previous
            // tile's sort, is behind this tile's barriers)
            uint32_t* const other = wcnt + (par ^ 1u) * nb;
            for (uint32_t i = tid; i < nb; i += BLOCK) other[i] = 0;
        }
        // chain protocol (k_scatter_chunked): digit d's run -> chunk ids -> wdesc[d]
        uint32_t bad = 0;
#pragma unroll
        for (int j = 0; j < DPT; j++) {
            if (!c[j]) continue;
            const uint32_t d = d0 + j;
            const uint32_t off = v0[j] % T, k0 = v0[j] / T, k1 = (v0[j] + c[j] - 1) / T;
            unsigned long long* tab = a.chunk_tab + (static_cast<size_t>(x) * nb + d) * a.maxch;
            auto take = [&]() -> uint32_t {
                const uint32_t r = atomicAdd(&tmp[17], 1u);
                if (r < 2) return tmp[16] + r;
                return id_lo + 2 * per + atomicAdd(pool, 1u);
            };
            auto publish = [&](uint32_t k, uint32_t id) {
                if (k >= a.maxch) return;   // flagged below
                __hip_atomic_store(&tab[k], kPublished | id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicMax(hints + d, (static_cast<unsigned long long>(k + 1) << 32) | id);
            };
            uint32_t id0 = id_lo, id1 = id_lo;
            if (off == 0) {
                id0 = take();
                publish(k0, id0);
            }
            if (k1 != k0) {
                id1 = take();
                publish(k1, id1);
            }
            if (k1 >= a.maxch) bad |= kChunkErrIndex;
            if (off != 0) {
                if ((hint[j] >> 32) == k0 + 1ull) {
                    id0 = static_cast<uint32_t>(hint[j]);
                } else if (k0 < a.maxch) {
                    unsigned long long v;
                    while (((v = __hip_atomic_load(&tab[k0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) == 0)
                        __builtin_amdgcn_s_sleep(2);
                    id0 = static_cast<uint32_t>(v);
                }
            }
            if (id0 < id_lo || id0 >= id_hi || id1 < id_lo || id1 >= id_hi) bad |= kChunkErrId;
            // sorted element k of digit d goes to chain slot v0 + (k - ds)
            const uint32_t split = ds[j] + (T - off);
            wdesc[d] = make_uint4(id0 * T + off - ds[j], id1 * T - split, split, 0u);
        }
        if (bad) {
            tmp[18] = 1;
            atomicOr(errw, bad);
        }
        __syncthreads();
        // sorted element k: code, digit, slot, all LDS reads of the ITEMS
        // elements in flight together; a lane past the tile (or every lane of
        // a tile with an id out of range) stores to its sink
        const uint32_t lim = tmp[18] ? 0u : cnt;
        auto write_out = [&](auto pow2) {
            int64_t v[ITEMS];
            uint32_t o[ITEMS];
#pragma unroll
            for (int i = 0; i < ITEMS; i++) v[i] = sbuf[i * BLOCK + tid];
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                const uint32_t k = i * BLOCK + tid;
                const uint4 w = wdesc[code_digit(static_cast<uint64_t>(v[i]), pow2)];
                o[i] = (k < w.z ? w.x : w.y) + k;
            }
#pragma unroll
            for (int i = 0; i < ITEMS; i++) *(i * BLOCK + tid < lim ? a.out_keys + o[i] : ssink) = v[i];
        };
        if (pow2q) write_out(std::true_type{});
        else write_out(std::false_type{});
        // the claim's registers stay live past the write-out: else they are
        // reused there, and a lane that issued no claim would first wait for
        // everything in flight (the compiler cannot tell which lanes did)
#pragma unroll
        for (int j = 0; j < DPT; j++) __asm__ volatile("" ::"v"(v0[j]), "v"(hint[j]));
        if (next >= t_end) return;
        tile = next;
        par ^= 1u;
    }
}

// ---------------------------------------------------------------------------
// Pipelined code pass (k_chunk_codes_pipe): k_chunk_codes with the claims of
// tile t resolved in the next iteration, beside the hashing and ranking of
// tile t + slots, so the cursor round trip is never waited for (one workgroup
// per CU spent ~1.5 us of every ~7 us tile on it). That needs chunk ids known
// before the runs that use them are resolved, so the chunks are
// PRE-ALLOCATED: chunks 0 and 1 of chain (x, d) are static, and the run that
// starts chunk j (the one holding its first slot) takes chunk j + 1's id and
// publishes it, with the chain's hint {j, id_j, id_j+1}; a run in chunk k
// finds id_k in the hint it loaded with its claim (hint chunk k or k - 1) and
// else in the chunk table, published one chunk earlier. A run's resolution
// waits only on claims strictly earlier in its chain (publishes first, then
// waits), so it always ends.
// Pool of shard x (pipe_pool_stride chunks): [0, 2 nb) chunks 0, 1 of each
// chain; then kPipeRes chunks per tile of the shard (the ids its starting
// runs take); then the shard's pool counter.
// ---------------------------------------------------------------------------
#ifndef PHJ_PIPE_RES   // (a measurement build may set another reservation)
#define PHJ_PIPE_RES 1
#endif
// (1: the pool's reservation per tile; chunks a tile starts beyond it come from
// the shard's pool counter. Measured against 3: S's pass +0.009 ms at C2, the
// pool 9.6 -> 4.8 GB and the LDS join's probe-side bound 1.02e9 -> 2.0e9 rows.)
constexpr uint32_t kPipeRes = PHJ_PIPE_RES;
__host__ __device__ constexpr uint32_t pipe_pool_stride(uint32_t per, uint32_t nb) {
    return 2 * nb + kPipeRes * per + per + nb + 1;
}
// hint word: chunk index j (20 bits) | id_j - pool base (22) | id_j+1 - pool base (22)
__device__ __forceinline__ unsigned long long pipe_hint(uint32_t j, uint32_t rid, uint32_t rid1) {
    return (static_cast<unsigned long long>(j) << 44) | (static_cast<unsigned long long>(rid) << 22) | rid1;
}

// LDS: two sorted tiles, two counter rows, ONE descriptor row (written between
// B2 and B3 for the previous tile, read by its write-out after B3; the next
// write is after the next B1 and B2), the scan / reservation words
__host__ __device__ constexpr size_t chunk_pipe_lds_bytes(int T, uint32_t nb) {
    return 2 * static_cast<size_t>(T) * 8 + (static_cast<size_t>(2 * nb + 3) / 4 * 4 + 4 * static_cast<size_t>(nb)) * 4 + 128;
}

// Registers: one workgroup per CU (LDS). WPE: waves per SIMD the registers
// must allow (0: the workgroup's own, BLOCK / 256; 1024 x 4 held to 5, <= 96
// VGPRs, spilled and ran 1.12 -> 1.54 ms at C2, so none is instantiated).
// PROF: thread 0's clock64 between the phases of each tile, summed per
// workgroup into a.prof: hash + rank, B1, scan,
// claims + B2, scatter + protocol, B3, write-out, then the tiles, and each
// wave's time from a barrier to the next (max / mean over the waves)
// (diagnostics; a barrier's time is wave 0's wait for the slowest wave).
template <int BLOCK, int ITEMS, int HK, int DPT = 1, int WPE = 0, bool PROF = false, int KPF = 1>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE ? WPE : BLOCK / 256)))
void k_chunk_codes_pipe(PassArgs a, uint32_t ntiles, uint32_t per) {
    constexpr int NW = BLOCK / 64;
    constexpr int T = BLOCK * ITEMS;
    static_assert(NW <= 16, "scan words [0, NW) below the reservation words");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t nb = a.nbins;   // host: nb <= DPT * BLOCK
    int64_t* sbuf = reinterpret_cast<int64_t*>(smem);                       // [2][T] sorted codes
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(sbuf + 2 * T);             // [2][nb] counter rows
    uint4* wdesc = reinterpret_cast<uint4*>(wcnt + (2 * nb + 3u) / 4 * 4);  // [nb] {k < split: slot - k, else, split}
    uint32_t* tmp = reinterpret_cast<uint32_t*>(wdesc + nb);                // [0, NW) scan; 16-19 reservations [2]; 20 bad tile

    const uint32_t x = blockIdx.x % a.nshards, slots = gridDim.x / a.nshards;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t t_end = min(ntiles, (x + 1) * per);
    uint32_t tile = x * per + blockIdx.x / a.nshards;
    if (tile >= t_end) return;
    const uint32_t wbase = wave * 64 * ITEMS;
    uint32_t* curs = a.chunk_cursor + static_cast<size_t>(x) * nb;
    uint32_t* pool = a.chunk_cursor + chunk_pool_word(nb, x);
    uint32_t* errw = a.chunk_cursor + chunk_err_word(nb);
    unsigned long long* hints = reinterpret_cast<unsigned long long*>(a.chunk_cursor + chunk_hint_word(nb)) + static_cast<size_t>(x) * nb;
    const uint32_t id_lo = x * a.pool_stride, id_hi = id_lo + a.pool_stride;
    const bool pow2q = a.f.mode == 0 && a.f.sub_bits == 0;
    // digit forms (workgroup-uniform): 2 = one bit-field extract (q = h mod a
    // power of two <= 2^32 and the digit's bits inside q), 1 = power of two, 0 = any plan
    const uint32_t dwidth = __popc(a.f.dmask);
    const int dform = pow2q && a.f.P <= (1ull << 32) && ((a.f.dmask + 1ull) & a.f.dmask) == 0 &&
                              ((static_cast<uint64_t>(a.f.dmask) << a.f.shift) & ~(a.f.P - 1)) == 0
                          ? 2
                          : pow2q ? 1 : 0;
    auto code_digit = [&](uint64_t h, auto form) -> uint32_t {
        if constexpr (decltype(form)::value == 2) return __builtin_amdgcn_ubfe(static_cast<uint32_t>(h), a.f.shift, dwidth);
        else if constexpr (decltype(form)::value == 1) return static_cast<uint32_t>((h & (a.f.P - 1)) >> a.f.shift) & a.f.dmask;
        else return static_cast<uint32_t>(q_from_hash(h, a.f) >> a.f.shift) & a.f.dmask;
    };
    using F0 = std::integral_constant<int, 0>;
    using F1 = std::integral_constant<int, 1>;
    using F2 = std::integral_constant<int, 2>;
    int64_t* const ssink = reinterpret_cast<int64_t*>(a.sink + static_cast<size_t>(blockIdx.x % kSinkGroups) * BLOCK + tid);
    __shared__ unsigned long long prof[PROF ? kP1ProfWords : 1];
    if (PROF && tid < kP1ProfWords) prof[tid] = 0;
    long long pc0 = 0;
    auto ptick = [&](int w) {
        if constexpr (PROF) {
            const long long now = clock64();
            if (tid == 0) prof[w] += static_cast<unsigned long long>(now - pc0);
            pc0 = now;
        }
    };
    // per wave: its clock from a barrier's exit to the next barrier's arrival,
    // max and mean over the waves (regions: B3 -> B1, B1 -> B2, B2 -> B3)
    __shared__ uint32_t parr[PROF ? 3 : 1][PROF ? NW : 1];
    long long px = 0;
    auto parrive = [&](int r) {
        if constexpr (PROF)
            if (lane == 0) parr[r][wave] = static_cast<uint32_t>(clock64() - px);
    };
    auto pexit = [&](int r) {
        if constexpr (PROF) {
            px = clock64();
            if (tid == 0) {
                uint32_t mx = 0;
                unsigned long long sm = 0;
                for (int w = 0; w < NW; w++) {
                    mx = max(mx, parr[r][w]);
                    sm += parr[r][w];
                }
                prof[8 + r] += mx;
                prof[11 + r] += sm / NW;
            }
        }
    };

    // KPF register buffers of keys used in turn (the loop unrolled KPF times,
    // so no register moves): tile t's keys were requested KPF tiles earlier
    int64_t key[KPF][ITEMS];
    const longlong2* rel = reinterpret_cast<const longlong2*>(a.in_keys);
    auto load = [&](int64_t* k, uint32_t t) {
        const uint32_t lo = t * T;
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t ix = min(lo + wbase + i * 64 + lane, a.n - 1);
            if (a.nt_load) k[i] = __builtin_nontemporal_load(&rel[ix].x);
            else k[i] = rel[ix].x;
        }
    };

    for (uint32_t i = tid; i < 2 * nb; i += BLOCK) wcnt[i] = 0;
#pragma unroll
    for (int f = 0; f < KPF; f++) {
        const uint32_t t = tile + f * slots;
        load(key[f], t < t_end ? t : tile);
    }
    {
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            __hip_atomic_store(ssink, 0ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __asm__ volatile("" ::: "memory");
        }
    }
    __syncthreads();
    // the previous tile's claims, resolved in this iteration
    // the claims' returns (cursor, hint) in two register sets, one per
    // iteration parity (the loop unrolled twice): a tile's claims land in set
    // cb and are read one iteration later as the previous tile's, with no
    // register move at the back edge (a move waits for its load, and vmcnt
    // retires in order: it would wait for the write-out's stores as well)
    uint32_t pc[DPT], pds[DPT], cv0[2][DPT];
    unsigned long long chint[2][DPT];
#pragma unroll
    for (int j = 0; j < DPT; j++) {
        pc[j] = 0;
        pds[j] = 0;
        cv0[0][j] = cv0[1][j] = 0;
        chint[0][j] = chint[1][j] = 0;
    }
    bool have_prev = false;
    uint32_t pcnt = 0, par = 0;
    const uint32_t d0 = tid * DPT;
    if (PROF) pc0 = px = clock64();
    auto iter = [&](auto kbc, auto cbc) -> bool {
        constexpr int kb = decltype(kbc)::value, cb = decltype(cbc)::value;
        uint32_t(&v0)[DPT] = cv0[cb];
        unsigned long long(&hint)[DPT] = chint[cb];
        const uint32_t(&pv0)[DPT] = cv0[cb ^ 1];
        const unsigned long long(&phint)[DPT] = chint[cb ^ 1];
        const bool live = tile < t_end;   // workgroup-uniform; false: the drain of the last tile
        uint32_t* const crow = wcnt + par * nb;
        const uint32_t cnt = live ? min(static_cast<uint32_t>(T), a.n - tile * T) : 0u;
        const uint32_t next = tile + slots;
        int64_t code[ITEMS];
        uint32_t dig[ITEMS], rank[ITEMS];
        if (live) {
            // full: a whole tile (every lane valid; the checks compiled out).
            // The loads stay outside the forms: one instance, straight into
            // the key buffer (a copy per form would be merged by register
            // moves, and a move waits for its load)
            auto hash_all = [&](auto form, auto full) {
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    const uint64_t h = hash64<HK>(static_cast<uint64_t>(key[kb][i]), a.f.seed);
                    code[i] = static_cast<int64_t>(h);
                    dig[i] = decltype(full)::value || wbase + i * 64 + lane < cnt ? code_digit(h, form) : 0u;
                }
            };
            if (dform == 2 && cnt == static_cast<uint32_t>(T)) hash_all(F2{}, std::true_type{});
            else if (dform == 2) hash_all(F2{}, std::false_type{});
            else if (dform == 1) hash_all(F1{}, std::false_type{});
            else hash_all(F0{}, std::false_type{});
            const uint32_t ahead = tile + KPF * slots;
            load(key[kb], ahead < t_end ? ahead : tile);
#pragma unroll
            for (int i = 0; i < ITEMS; i++) rank[i] = atomicAdd(&crow[dig[i]], wbase + i * 64 + lane < cnt ? 1u : 0u);
        }
        ptick(0);
        parrive(0);
        __syncthreads();   // B1: ranks counted
        ptick(1);
        pexit(0);
        uint32_t c[DPT], ds[DPT];
        {
            uint32_t local = 0;
#pragma unroll
            for (int j = 0; j < DPT; j++) {
                c[j] = live && d0 + j < nb ? crow[d0 + j] : 0u;
                local += c[j];
            }
            uint32_t total;
            uint32_t run = block_exclusive_scan_t<NW, false>(local, tmp, total);
#pragma unroll
            for (int j = 0; j < DPT; j++) {
                ds[j] = run;
                if (live && d0 + j < nb) crow[d0 + j] = run;
                run += c[j];
            }
            ptick(2);
            if (live) {   // claims of every digit (0 adds too): resolved next iteration
                // (a thread past the plan's digits claims 0 from its own sink word:
                // with fewer digits than threads, clamping them onto the last digit
                // serialised up to 768 returning atomics per tile on one cursor)
#pragma unroll
                for (int j = 0; j < DPT; j++) {
                    const bool real = d0 + j < nb;
                    uint32_t* cw = real ? curs + d0 + j : reinterpret_cast<uint32_t*>(ssink);
                    unsigned long long* hw = real ? hints + d0 + j : reinterpret_cast<unsigned long long*>(ssink);
                    v0[j] = atomicAdd(cw, real ? c[j] : 0u);
                    hint[j] = __hip_atomic_load(hw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (tid == 0) {
                if (live) {
                    tmp[16 + 2 * par] = id_lo + 2 * nb + kPipeRes * (tile - x * per);   // this tile's reserved chunks
                    tmp[17 + 2 * par] = 0;
                }
                tmp[20] = 0;
            }
        }
        parrive(1);
        __syncthreads();   // B2: tile-local starts, reservations
        ptick(3);
        pexit(1);
        if (live) {
            uint32_t base[ITEMS];
#pragma unroll
            for (int i = 0; i < ITEMS; i++) base[i] = crow[dig[i]];
#pragma unroll
            for (int i = 0; i < ITEMS; i++)
                if (wbase + i * 64 + lane < cnt) sbuf[par * T + base[i] + rank[i]] = code[i];
        }
        const uint32_t pp = par ^ 1u;   // the previous tile's buffers
        // the next tile's counter row: the previous tile's, no longer read
        for (uint32_t i = tid; i < nb; i += BLOCK) wcnt[pp * nb + i] = 0;
        if (have_prev) {
            uint32_t bad = 0;
            uint32_t st[DPT], nid[DPT];   // chunk this run starts (or ~0u) and the id it took for st + 1
            // phase 1: publish (no waits)
#pragma unroll
            for (int j = 0; j < DPT; j++) {
                st[j] = 0xffffffffu;
                nid[j] = 0;
                if (!pc[j]) continue;
                const uint32_t d = d0 + j;
                const uint32_t off = pv0[j] % T, k0 = pv0[j] / T, k1 = (pv0[j] + pc[j] - 1) / T;
                if (off == 0) st[j] = k0;
                else if (k1 != k0) st[j] = k1;
                if (st[j] == 0xffffffffu) continue;
                unsigned long long* tab = a.chunk_tab + (static_cast<size_t>(x) * nb + d) * a.maxch;
                const uint32_t s0 = id_lo + 2 * d;   // static chunks 0, 1 of the chain
                if (st[j] == 0) {
                    nid[j] = s0 + 1;
                    if (a.maxch >= 2) {
                        __hip_atomic_store(&tab[0], kPublished | s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&tab[1], kPublished | (s0 + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } else {
                        bad |= kChunkErrIndex;
                    }
                } else {
                    const uint32_t r = atomicAdd(&tmp[17 + 2 * pp], 1u);
                    nid[j] = r < kPipeRes ? tmp[16 + 2 * pp] + r : id_lo + 2 * nb + kPipeRes * per + atomicAdd(pool, 1u);
                    // (a chain's last possible chunk needs no successor)
                    if (st[j] + 1 < a.maxch)
                        __hip_atomic_store(&tab[st[j] + 1], kPublished | nid[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            // phase 2: resolve the ids of the chunks each run writes
#pragma unroll
            for (int j = 0; j < DPT; j++) {
                if (!pc[j]) continue;
                const uint32_t d = d0 + j;
                const uint32_t off = pv0[j] % T, k0 = pv0[j] / T, k1 = (pv0[j] + pc[j] - 1) / T;
                unsigned long long* tab = a.chunk_tab + (static_cast<size_t>(x) * nb + d) * a.maxch;
                const uint32_t s0 = id_lo + 2 * d;
                const uint32_t hk = static_cast<uint32_t>(phint[j] >> 44);
                const uint32_t hid = phint[j] ? id_lo + (static_cast<uint32_t>(phint[j] >> 22) & 0x3fffffu) : s0;
                const uint32_t hid1 = phint[j] ? id_lo + (static_cast<uint32_t>(phint[j]) & 0x3fffffu) : s0 + 1;
                auto id_of = [&](uint32_t k) -> uint32_t {
                    if (k == 0) return s0;
                    if (k == 1) return s0 + 1;
                    if (k == hk) return hid;
                    if (k == hk + 1) return hid1;
                    if (k >= a.maxch) {
                        bad |= kChunkErrIndex;
                        return id_lo;
                    }
                    unsigned long long v;
                    while (((v = __hip_atomic_load(&tab[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) == 0)
                        __builtin_amdgcn_s_sleep(2);
                    return static_cast<uint32_t>(v);
                };
                const uint32_t id0 = id_of(k0);
                const uint32_t id1 = k1 != k0 ? id_of(k1) : id0;
                if (st[j] != 0xffffffffu && st[j] != 0) {
                    const uint32_t ids = st[j] == k0 ? id0 : id1;
                    atomicMax(hints + d, pipe_hint(st[j], ids - id_lo, nid[j] - id_lo));
                }
                if (id0 < id_lo || id0 >= id_hi || id1 < id_lo || id1 >= id_hi || nid[j] >= id_hi) bad |= kChunkErrId;
                const uint32_t split = pds[j] + (T - off);
                wdesc[d] = make_uint4(id0 * T + off - pds[j], id1 * T - split, split, 0u);
            }
            if (bad) {
                tmp[20] = 1;
                atomicOr(errw, bad);
            }
        }
        ptick(4);
        parrive(2);
        __syncthreads();   // B3: the previous tile's slots, this tile sorted
        ptick(5);
        pexit(2);
        if (have_prev) {
            const uint32_t lim = tmp[20] ? 0u : pcnt;
            auto write_out = [&](auto form, auto full) {
                int64_t v[ITEMS];
                uint32_t o[ITEMS];
#pragma unroll
                for (int i = 0; i < ITEMS; i++) v[i] = sbuf[pp * T + i * BLOCK + tid];
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    const uint32_t k = i * BLOCK + tid;
                    const uint4 w = wdesc[code_digit(static_cast<uint64_t>(v[i]), form)];
                    o[i] = (k < w.z ? w.x : w.y) + k;
                }
#pragma unroll
                for (int i = 0; i < ITEMS; i++) {
                    if constexpr (decltype(full)::value) a.out_keys[o[i]] = v[i];
                    else *(i * BLOCK + tid < lim ? a.out_keys + o[i] : ssink) = v[i];
                }
            };
            if (dform == 2 && lim == static_cast<uint32_t>(T)) write_out(F2{}, std::true_type{});
            else if (dform == 2) write_out(F2{}, std::false_type{});
            else if (dform == 1) write_out(F1{}, std::false_type{});
            else write_out(F0{}, std::false_type{});
        }
        ptick(6);
        if (PROF && tid == 0) prof[PROF ? 7 : 0] += 1;
        if (!live) {
            if (PROF && tid == 0 && a.prof)
                for (int w = 0; w < kP1ProfWords; w++) atomicAdd(&a.prof[w], prof[PROF ? w : 0]);
            return false;
        }
#pragma unroll
        for (int j = 0; j < DPT; j++) {
            pc[j] = c[j];
            pds[j] = ds[j];
        }
        pcnt = cnt;
        have_prev = true;
        tile = next;
        par ^= 1u;
        return true;
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    static_assert(KPF == 1 || KPF == 2, "one or two tiles of keys in flight");
    if constexpr (KPF == 1) {
        while (iter(I0{}, I0{}) && iter(I0{}, I1{})) {
        }
    } else {
        while (iter(I0{}, I0{}) && iter(I1{}, I1{})) {
        }
    }
}

constexpr int kScanItems = 16;
constexpr int kScanBlockElems = kBlock * kScanItems;  // 4096

struct ScanArgs {
    uint32_t* data;       // narrays arrays at stride `stride`
    uint32_t* partials;   // narrays * nblk
    uint32_t len;
    uint32_t stride;
    uint32_t nblk;
    uint32_t pad;
};

__global__ __launch_bounds__(kBlock) void k_scan_reduce(ScanArgs s) {
    __shared__ uint32_t tmp[16];
    const uint32_t* d = s.data + static_cast<size_t>(blockIdx.y) * s.stride;
    const uint32_t base = blockIdx.x * kScanBlockElems;
    uint32_t acc = 0;
    if (base + kScanBlockElems <= s.len && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
        const uint4* q = reinterpret_cast<const uint4*>(d + base);   // 16 B per lane, coalesced
#pragma unroll
        for (int i = 0; i < kScanItems / 4; i++) {
            const uint4 v = q[i * kBlock + threadIdx.x];
            acc += v.x + v.y + v.z + v.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kScanItems; i++) {
            const uint32_t idx = base + i * kBlock + threadIdx.x;
            if (idx < s.len) acc += d[idx];
        }
    }
    uint32_t total;
    block_exclusive_scan(acc, tmp, total);
    if (threadIdx.x == 0) s.partials[blockIdx.y * s.nblk + blockIdx.x] = total;
}

// k_scan_apply: per block, exclusive scan of its elements plus the sum of all
// preceding blocks' partials (read directly; no separate partials-scan kernel).
__global__ __launch_bounds__(kBlock) void k_scan_apply(ScanArgs s) {
    __shared__ uint32_t tmp[16];
    uint32_t* d = s.data + static_cast<size_t>(blockIdx.y) * s.stride;
    const uint32_t base = blockIdx.x * kScanBlockElems + threadIdx.x * kScanItems;
    const bool vec = (reinterpret_cast<uintptr_t>(d) & 15) == 0 && base + kScanItems <= s.len;
    uint32_t v[kScanItems];
    uint32_t acc = 0;
    if (vec) {
        const uint4* q = reinterpret_cast<const uint4*>(d + base);
#pragma unroll
        for (int i = 0; i < kScanItems / 4; i++) {
            const uint4 t = q[i];
            v[4 * i] = t.x;
            v[4 * i + 1] = t.y;
            v[4 * i + 2] = t.z;
            v[4 * i + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kScanItems; i++) {
            const uint32_t idx = base + i;
            v[i] = idx < s.len ? d[idx] : 0u;
        }
    }
#pragma unroll
    for (int i = 0; i < kScanItems; i++) acc += v[i];
    // prefix of the preceding blocks' sums (L2-resident, <= a few thousand words)
    __shared__ uint32_t pre;
    {
        const uint32_t* pp = s.partials + blockIdx.y * s.nblk;
        uint32_t x = 0;
        for (uint32_t i = threadIdx.x; i < blockIdx.x; i += kBlock) x += pp[i];
        uint32_t t;
        block_exclusive_scan(x, tmp, t);
        if (threadIdx.x == 0) pre = t;
        __syncthreads();
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(acc, tmp, total) + pre;
    if (vec) {
        uint4* q = reinterpret_cast<uint4*>(d + base);
#pragma unroll
        for (int i = 0; i < kScanItems / 4; i++) {
            uint4 t;
            t.x = run;
            run += v[4 * i];
            t.y = run;
            run += v[4 * i + 1];
            t.z = run;
            run += v[4 * i + 2];
            t.w = run;
            run += v[4 * i + 3];
            q[i] = t;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kScanItems; i++) {
            const uint32_t idx = base + i;
            if (idx < s.len) d[idx] = run;
            run += v[i];
        }
    }
}

// ---------------------------------------------------------------------------
// Pass bookkeeping.
// ---------------------------------------------------------------------------
// The single-workgroup bookkeeping kernels below use kFinBlock threads and
// loop over the digits: a 1024-thread workgroup needs 16 wave slots on ONE CU,
// which a persistent pass beside it (S's pass 1, two workgroups per CU) may not
// leave free anywhere, so R's chain would stall behind it (measured 0.75 ms).
constexpr uint32_t kFinBlock = 256;

// Exclusive scan over the block with a running carry (kFinBlock threads).
template <uint32_t NT = kFinBlock>
__device__ __forceinline__ uint32_t fin_block_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < NT / 64; w++) {
        const uint32_t t = wsum[w];
        if (w < wave) before += t;
        all += t;
    }
    __syncthreads();
    total = all;
    return before + x - v;
}

// After pass 1 (single segment): bounds1[d] for d <= nb1 and, for a second
// pass, the per-segment cumulative tile counts.
__global__ __launch_bounds__(kFinBlock) void k_pass1_finish(const uint32_t* hist, uint32_t ntiles,
                                                            uint32_t nb, uint32_t n, uint32_t T,
                                                            uint32_t* bounds1, uint32_t* tile_base2) {
    __shared__ uint32_t wsum[kFinBlock / 64];
    const uint32_t tid = threadIdx.x;
    for (uint32_t d = tid; d < nb; d += kFinBlock) bounds1[d] = ntiles ? hist[static_cast<size_t>(d) * ntiles] : 0u;
    if (tid == 0) bounds1[nb] = n;
    __syncthreads();
    if (tile_base2 == nullptr) return;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nb; base += kFinBlock) {
        const uint32_t d = base + tid;
        const uint32_t v = d < nb ? (bounds1[d + 1] - bounds1[d] + T - 1) / T : 0u;
        uint32_t all;
        const uint32_t ex = fin_block_scan(v, wsum, all);
        if (d < nb) tile_base2[d] = carry + ex;
        carry += all;
    }
    if (tid == 0) tile_base2[nb] = carry;
}

// tile_seg[t] = s for every tile t of segment s (one wave per segment).
__global__ __launch_bounds__(kBlock) void k_tile_seg(const uint32_t* tile_base, uint32_t nseg,
                                                     uint32_t* tile_seg) {
    const uint32_t s = blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (s >= nseg) return;
    const uint32_t lo = tile_base[s], hi = tile_base[s + 1];
    for (uint32_t t = lo + (threadIdx.x & 63); t < hi; t += 64) tile_seg[t] = s;
}

// Chunked pass-1 output: segment s's tiles are the chunks of its nshards
// chains, shard by shard, chunk by chunk: tile_seg / tile_start (first slot) /
// tile_cnt (tuples) of each. One wave per chain (segment s, shard x): lane x'
// reads chain (s, x')'s size for the chain's first tile, then the lanes write
// the chain's chunks. An entry that is not published or names a chunk outside
// shard x's pool (a stale table) becomes an empty tile and sets the pass's
// error word (the consumers read no slot through it). Entry nch (the chunk
// k_chunk_codes_pipe pre-allocates after a chain's last one) is cleared too.
__global__ __launch_bounds__(kBlock) void k_tile_chunks(const uint32_t* tile_base, uint32_t* sizes,
                                                        uint32_t nseg, uint32_t nshards,
                                                        unsigned long long* chunk_tab, uint32_t maxch,
                                                        uint32_t pool_stride, uint32_t T, uint32_t* tile_seg,
                                                        uint32_t* tile_start, uint32_t* tile_cnt) {
    const uint32_t w = blockIdx.x * kWaves + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= nseg * nshards) return;
    const uint32_t s = w / nshards, x = w - s * nshards;
    const uint32_t z = lane < x ? sizes[lane * nseg + s] : 0u;   // chains before x in this segment
    uint32_t before = (z + T - 1) / T;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) before += __shfl_xor(before, o, 64);
    const uint32_t szx = sizes[x * nseg + s], nch = (szx + T - 1) / T;
    const uint32_t t0 = tile_base[s] + before;
    unsigned long long* tab = chunk_tab + (static_cast<size_t>(x) * nseg + s) * maxch;
    uint32_t bad = 0;
    for (uint32_t k = lane; k < nch; k += 64) {
        const unsigned long long v = k < maxch ? tab[k] : 0ull;
        const uint32_t id = static_cast<uint32_t>(v);
        const bool ok = k < maxch && (v >> 32) == 1ull && id >= x * pool_stride && id < (x + 1) * pool_stride;
        tile_seg[t0 + k] = s;
        tile_start[t0 + k] = ok ? id * T : 0u;
        tile_cnt[t0 + k] = ok ? min(T, szx - k * T) : 0u;
        if (!ok) bad |= kChunkErrTable;
        if (k < maxch) tab[k] = 0;   // the next pass starts from an all-zero table (kPublished)
    }
    // the pipelined pass pre-allocates the chunk after a chain's last one
    if (lane == 0 && nch < maxch) tab[nch] = 0;
    if (bad) atomicOr(sizes + chunk_err_word(nseg), bad);
}

// After a chunked pass 1: bounds1 = exclusive scan of the digit sizes (summed
// over the shards: the segments' offsets in the pass-2 output) and
// tile_base2 = exclusive scan of their chunk counts; `zero` (may be null: four
// words) and `clr` (may be null: clr16 16-B words, another pass's chunk state)
// are cleared. One workgroup.
constexpr uint32_t kFinSizesBlock = 1024;   // one digit per thread at 1024 clusters: one round of shard loads
__global__ __launch_bounds__(kFinSizesBlock) void k_pass1_finish_sizes(const uint32_t* sizes, uint32_t nb, uint32_t nshards,
                                                                       uint32_t n, uint32_t T, uint32_t* bounds1,
                                                                       uint32_t* tile_base2, unsigned long long* zero,
                                                                       uint4* clr, uint32_t clr16) {
    constexpr uint32_t B = kFinSizesBlock;
    __shared__ uint32_t wsum[2][B / 64];
    const uint32_t tid = threadIdx.x;
    if (zero && tid < 4) zero[tid] = 0;   // the on-chip probe's {count, failed} and its clock split (one launch fewer before it)
    if (clr)
        for (uint32_t i = tid; i < clr16; i += B) clr[i] = make_uint4(0, 0, 0, 0);
    uint32_t cx = 0, cy = 0;
    for (uint32_t base = 0; base < nb; base += B) {
        const uint32_t d = base + tid;
        uint32_t z[kShards];
#pragma unroll
        for (uint32_t x = 0; x < kShards; x++) z[x] = d < nb && x < nshards ? sizes[x * nb + d] : 0u;   // all in flight
        uint32_t v = 0, t = 0;
#pragma unroll
        for (uint32_t x = 0; x < kShards; x++) {
            v += z[x];
            t += (z[x] + T - 1) / T;
        }
        uint32_t ax, ay;
        const uint32_t ex = fin_block_scan<B>(v, wsum[0], ax);
        const uint32_t ey = fin_block_scan<B>(t, wsum[1], ay);
        if (d < nb) {
            bounds1[d] = cx + ex;
            tile_base2[d] = cy + ey;
        }
        cx += ax;
        cy += ay;
    }
    if (tid == 0) {
        bounds1[nb] = n;
        tile_base2[nb] = cy;
    }
}

// Final bounds after a segmented pass 2: bounds[s * nb2 + d].
__global__ __launch_bounds__(kBlock) void k_pass2_bounds(const uint32_t* hist2,
                                                         const uint32_t* tile_base2,
                                                         const uint32_t* bounds1, uint32_t nb1,
                                                         uint32_t nb2, uint32_t n,
                                                         uint32_t* bounds) {
    const uint32_t P = nb1 * nb2;
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i > P) return;
    if (i == P) {
        bounds[P] = n;
        return;
    }
    const uint32_t s = i / nb2, d = i - s * nb2;
    const uint32_t tb = tile_base2[s], nt = tile_base2[s + 1] - tb;
    bounds[i] = nt ? hist2[static_cast<size_t>(tb) * nb2 + static_cast<size_t>(d) * nt] : bounds1[s];
}

}  // namespace phj
