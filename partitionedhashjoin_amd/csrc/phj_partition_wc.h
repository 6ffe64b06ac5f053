// phj_partition_wc.h — partition pass with software write-combining (SWWC).
//
// Same stable partition as k_scatter (identical output layout), restructured
// for HBM efficiency:
//   * one workgroup owns a SUPER-tile of K sub-tiles (K * 256 * ITEMS tuples),
//     so the histogram has one row per super-tile (K x fewer rows to write and
//     scan than per-tile rows);
//   * every sub-tile is sorted by digit in LDS (stable wave-match ranking), then
//     each digit's run is appended to a per-digit LDS line buffer of LW
//     elements per column; only COMPLETE, LW-aligned lines go to HBM (16
//     lanes x 8 B = one 128-B line for LW = 16), so neighbouring workgroups
//     never write the same line except at the two ends of a run;
//   * the next sub-tile's tuples are loaded into registers while the current
//     one is being written out.
// Limits: nbins <= 256 (one digit per thread in the per-digit phases).
#pragma once

#include "phj_partition.h"

namespace phj {

constexpr int kWcMaxBins = 256;

// Per-super-tile digit histogram -> hist[(tb_s * nbins) + d * ntiles_s + tseg].
template <int ITEMS, bool AOS, int HK>
__global__ __launch_bounds__(kBlock) void k_hist_super(PassArgs a, uint32_t tsz) {
    constexpr uint32_t T = kBlock * ITEMS;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(smem);  // [kWaves][nbins]
    TileLoc L;
    if (!locate_tile_rt(a, tile_id(a), tsz, L)) return;
    const uint32_t nb = a.nbins;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (uint32_t i = tid; i < kWaves * nb; i += kBlock) wcnt[i] = 0;
    __syncthreads();
    uint32_t* my = wcnt + wave * nb;
    const uint32_t wbase = wave * 64 * ITEMS;
    for (uint32_t base = L.lo; base < L.hi; base += T) {
        const uint32_t cnt = min(T, L.hi - base);
        int64_t key[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = wbase + i * 64 + lane;
            key[i] = 0;
            if (e < cnt) {
                if constexpr (AOS) key[i] = reinterpret_cast<const longlong2*>(a.in_keys)[base + e].x;
                else key[i] = a.in_keys[base + e];
            }
        }
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = wbase + i * 64 + lane;
            const bool valid = e < cnt;
            const uint32_t d = valid ? digit_of<HK>(static_cast<uint64_t>(key[i]), a.f) : 0u;
            const uint64_t peers = match_digit(d, valid, a.nbits);
            if (valid && (peers & lanemask_lt()) == 0) my[d] += __popcll(peers);
        }
    }
    __syncthreads();
    uint32_t* out = a.hist + static_cast<size_t>(L.tb_s) * nb + L.tseg;
    for (uint32_t d = tid; d < nb; d += kBlock) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) c += wcnt[w * nb + d];
        out[static_cast<size_t>(d) * L.ntiles_s] = c;
    }
}

__host__ __device__ constexpr size_t scatter_wc_lds_bytes(int T, int LW) {
    // skey/spay 16T | line buffers 16*256*LW | wcnt 4*kWaves*256 | 7 x 256 u32 | tmp 64 | line map
    return static_cast<size_t>(T) * 16 + static_cast<size_t>(16) * kWcMaxBins * LW +
           static_cast<size_t>(4) * kWaves * kWcMaxBins + 7 * 4 * kWcMaxBins + 64 +
           2 * (static_cast<size_t>(T) + kWcMaxBins);
}

template <int ITEMS, bool AOS, int HK, int LW>
__global__ __launch_bounds__(kBlock) void k_scatter_wc(PassArgs a, uint32_t tsz) {
    constexpr uint32_t T = kBlock * ITEMS;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t nb = a.nbins;
    int64_t* skey = reinterpret_cast<int64_t*>(smem);
    int64_t* spay = skey + T;
    int64_t* wbk = spay + T;                                   // [256][LW]
    int64_t* wbp = wbk + kWcMaxBins * LW;                      // [256][LW]
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(wbp + kWcMaxBins * LW);  // [kWaves][nb]
    uint32_t* dstart = wcnt + kWaves * kWcMaxBins;
    uint32_t* dcnt = dstart + kWcMaxBins;
    uint32_t* cur = dcnt + kWcMaxBins;      // next global slot of this workgroup per digit
    uint32_t* start = cur + kWcMaxBins;     // first global slot of this workgroup per digit
    uint32_t* flin = start + kWcMaxBins;    // first line touched by this sub-tile
    uint32_t* lbase = flin + kWcMaxBins;    // exclusive scan of complete lines per digit
    uint32_t* misc = lbase + kWcMaxBins;    // [0] = total lines
    uint32_t* tmp = misc + kWcMaxBins;      // 16 words
    uint16_t* ldig = reinterpret_cast<uint16_t*>(tmp + 16);   // line -> digit

    TileLoc L;
    if (!locate_tile_rt(a, tile_id(a), tsz, L)) return;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    {
        const uint32_t* h = a.hist + static_cast<size_t>(L.tb_s) * nb + L.tseg;
        for (uint32_t d = tid; d < nb; d += kBlock) {
            const uint32_t o = h[static_cast<size_t>(d) * L.ntiles_s];
            cur[d] = o;
            start[d] = o;
        }
    }
    const uint32_t wbase = wave * 64 * ITEMS;
    int64_t key[ITEMS], pay[ITEMS];
    {
        const uint32_t cnt = min(T, L.hi - L.lo);
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = wbase + i * 64 + lane;
            key[i] = 0;
            pay[i] = 0;
            if (e < cnt) load_tuple<AOS>(a, L.lo + e, key[i], pay[i]);
        }
    }
    uint32_t* my = wcnt + wave * nb;
    for (uint32_t base = L.lo; base < L.hi; base += T) {
        const uint32_t cnt = min(T, L.hi - base);
        for (uint32_t i = tid; i < kWaves * nb; i += kBlock) wcnt[i] = 0;
        __syncthreads();
        // (1) stable rank inside the sub-tile
        uint32_t dig[ITEMS], rank[ITEMS];
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
        // (2) digit starts inside the sub-tile; per-wave starts
        {
            uint32_t tot = 0;
            if (tid < nb) {
#pragma unroll
                for (int w = 0; w < kWaves; w++) tot += wcnt[w * nb + tid];
            }
            uint32_t all;
            uint32_t run = block_exclusive_scan(tot, tmp, all);
            if (tid < nb) {
                dstart[tid] = run;
                dcnt[tid] = tot;
#pragma unroll
                for (int w = 0; w < kWaves; w++) {
                    const uint32_t c = wcnt[w * nb + tid];
                    wcnt[w * nb + tid] = run;
                    run += c;
                }
            }
        }
        __syncthreads();
        // (3) place the sub-tile in LDS in digit order
#pragma unroll
        for (int i = 0; i < ITEMS; i++) {
            const uint32_t e = wbase + i * 64 + lane;
            if (e < cnt) {
                const uint32_t pos = my[dig[i]] + rank[i];
                skey[pos] = key[i];
                spay[pos] = pay[i];
            }
        }
        // (4) prefetch the next sub-tile while this one is written out
        {
            const uint32_t nbase = base + T;
            const uint32_t ncnt = nbase < L.hi ? min(T, L.hi - nbase) : 0u;
#pragma unroll
            for (int i = 0; i < ITEMS; i++) {
                const uint32_t e = wbase + i * 64 + lane;
                if (e < ncnt) load_tuple<AOS>(a, nbase + e, key[i], pay[i]);
            }
        }
        // (5) complete lines per digit
        {
            uint32_t nl = 0;
            if (tid < nb) {
                const uint32_t lo = cur[tid], hi = lo + dcnt[tid];
                flin[tid] = lo / LW;
                nl = hi / LW - lo / LW;
            }
            uint32_t total;
            const uint32_t lb = block_exclusive_scan(nl, tmp, total);  // (barriers inside)
            if (tid < nb) {
                lbase[tid] = lb;
                for (uint32_t k = 0; k < nl; k++) ldig[lb + k] = static_cast<uint16_t>(tid);
            }
            if (tid == 0) misc[0] = total;
        }
        __syncthreads();
        // (6) write complete lines: LW consecutive lanes store one aligned line per column
        {
            const uint32_t nelem = misc[0] * LW;
            for (uint32_t idx = tid; idx < nelem; idx += kBlock) {
                const uint32_t l = idx / LW, j = idx % LW;
                const uint32_t d = ldig[l];
                const uint32_t g = (flin[d] + (l - lbase[d])) * LW + j;
                const uint32_t lo = cur[d];
                int64_t k, p;
                bool write = true;
                if (g >= lo) {
                    const uint32_t s = dstart[d] + (g - lo);
                    k = skey[s];
                    p = spay[s];
                } else {
                    write = g >= start[d];   // older slots of the line belong to another workgroup
                    k = wbk[d * LW + j];
                    p = wbp[d * LW + j];
                }
                if (write) {
                    a.out_keys[g] = k;
                    a.out_pays[g] = p;
                }
            }
        }
        __syncthreads();
        // (7) keep the incomplete tail line of every digit in its buffer
        if (tid < nb) {
            const uint32_t lo = cur[tid], hi = lo + dcnt[tid];
            const uint32_t tail = hi / LW * LW;
            for (uint32_t g = tail > lo ? tail : lo; g < hi; g++) {
                const uint32_t s = dstart[tid] + (g - lo);
                wbk[tid * LW + (g % LW)] = skey[s];
                wbp[tid * LW + (g % LW)] = spay[s];
            }
            cur[tid] = hi;
        }
        __syncthreads();
    }
    // flush the partial tail lines (valid slots only)
    for (uint32_t idx = tid; idx < nb * LW; idx += kBlock) {
        const uint32_t d = idx / LW, j = idx % LW;
        const uint32_t c = cur[d];
        const uint32_t g = c / LW * LW + j;
        if (g < c && g >= start[d]) {
            a.out_keys[g] = wbk[d * LW + j];
            a.out_pays[g] = wbp[d * LW + j];
        }
    }
}

}  // namespace phj
