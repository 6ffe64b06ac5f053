// Bandwidth ceilings on MI355X for the partition pass's access patterns.
// Standalone: hipcc --offload-arch=gfx950 -O3 -o membw scripts/membw.hip
//   copy16      : 16 B / lane streaming copy (tile of BLOCK*ITEMS tuples per block)
//   read16      : 16 B / lane streaming read (sum)
//   write16     : 16 B / lane streaming store
//   runs_soa    : read a tile of AoS tuples, write key / payload columns into
//                 R runs per tile at the partitioned layout (the scatter's write
//                 pattern with uniform digits, no LDS ranking)
//   runs_aos    : same with 16-B AoS output
//   *_nt        : nontemporal stores
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

template <int BLOCK, int ITEMS, bool NT>
__global__ __launch_bounds__(BLOCK) void k_copy16(const longlong2* __restrict__ in, longlong2* __restrict__ out,
                                                  size_t n) {
    const size_t base = static_cast<size_t>(blockIdx.x) * BLOCK * ITEMS;
    longlong2 v[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const size_t e = base + i * BLOCK + threadIdx.x;
        if (e < n) v[i] = in[e];
    }
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const size_t e = base + i * BLOCK + threadIdx.x;
        if (e < n) {
            if constexpr (NT) {
                __builtin_nontemporal_store(v[i].x, &out[e].x);
                __builtin_nontemporal_store(v[i].y, &out[e].y);
            } else {
                out[e] = v[i];
            }
        }
    }
}

template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_read16(const longlong2* __restrict__ in, unsigned long long* sink,
                                                  size_t n) {
    const size_t base = static_cast<size_t>(blockIdx.x) * BLOCK * ITEMS;
    long long acc = 0;
    longlong2 v[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const size_t e = base + i * BLOCK + threadIdx.x;
        v[i] = e < n ? in[e] : make_longlong2(0, 0);
    }
#pragma unroll
    for (int i = 0; i < ITEMS; i++) acc += v[i].x ^ v[i].y;
    if (acc == 0x7fffffffffffffffll) atomicAdd(sink, 1ull);
}

template <int BLOCK, int ITEMS, bool NT>
__global__ __launch_bounds__(BLOCK) void k_write16(longlong2* __restrict__ out, size_t n) {
    const size_t base = static_cast<size_t>(blockIdx.x) * BLOCK * ITEMS;
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const size_t e = base + i * BLOCK + threadIdx.x;
        if (e < n) {
            if constexpr (NT) {
                __builtin_nontemporal_store((long long)e, &out[e].x);
                __builtin_nontemporal_store((long long)i, &out[e].y);
            } else {
                out[e] = make_longlong2(e, i);
            }
        }
    }
}

// Tile t of T tuples holds R runs of T/R tuples (run r = digit r); the output
// of digit r is a contiguous partition of n/R tuples, tile t's run at t*T/R.
template <int BLOCK, int ITEMS, bool AOS_OUT, bool NT, bool REMAP>
__global__ __launch_bounds__(BLOCK) void k_runs(const longlong2* __restrict__ in, long long* __restrict__ ok,
                                                long long* __restrict__ op, size_t n, int R) {
    constexpr int T = BLOCK * ITEMS;
    uint32_t tile = blockIdx.x;
    if (REMAP) {
        const uint32_t g = gridDim.x;
        if ((g & 7) == 0) tile = (blockIdx.x & 7) * (g >> 3) + (blockIdx.x >> 3);
    }
    const size_t base = static_cast<size_t>(tile) * T;
    const size_t ntiles = gridDim.x;
    const int run = T / R;
    const size_t plen = ntiles * run;
    longlong2 v[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; i++) v[i] = in[base + i * BLOCK + threadIdx.x];
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const uint32_t k = i * BLOCK + threadIdx.x;
        const uint32_t d = k / run;
        const size_t o = d * plen + static_cast<size_t>(tile) * run + (k - d * run);
        if constexpr (AOS_OUT) {
            longlong2* o2 = reinterpret_cast<longlong2*>(ok);
            if constexpr (NT) {
                __builtin_nontemporal_store(v[i].x, &o2[o].x);
                __builtin_nontemporal_store(v[i].y, &o2[o].y);
            } else {
                o2[o] = v[i];
            }
        } else {
            if constexpr (NT) {
                __builtin_nontemporal_store(v[i].x, &ok[o]);
                __builtin_nontemporal_store(v[i].y, &op[o]);
            } else {
                ok[o] = v[i].x;
                op[o] = v[i].y;
            }
        }
    }
}

// Histogram write shapes: each wave writes one tile's nb counters, either as a
// column of the [digit][tile] layout (stride ntiles) or a row of [tile][digit].
template <bool COLUMN, bool REMAP>
__global__ __launch_bounds__(256) void k_histw(uint32_t* out, uint32_t ntiles, uint32_t nb) {
    uint32_t b = blockIdx.x;
    if (REMAP) {
        const uint32_t g = gridDim.x;
        if ((g & 7) == 0) b = (blockIdx.x & 7) * (g >> 3) + (blockIdx.x >> 3);
    }
    const uint32_t tile = b * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (tile >= ntiles) return;
    for (uint32_t d = lane; d < nb; d += 64) {
        if (COLUMN) out[static_cast<size_t>(d) * ntiles + tile] = d ^ tile;
        else out[static_cast<size_t>(tile) * nb + d] = d ^ tile;
    }
}

// The same counters read back per tile (the scatter's offset load).
template <bool COLUMN, bool REMAP>
__global__ __launch_bounds__(256) void k_histr(const uint32_t* in, uint32_t ntiles, uint32_t nb,
                                              unsigned long long* sink) {
    uint32_t b = blockIdx.x;
    if (REMAP) {
        const uint32_t g = gridDim.x;
        if ((g & 7) == 0) b = (blockIdx.x & 7) * (g >> 3) + (blockIdx.x >> 3);
    }
    const uint32_t tile = b * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (tile >= ntiles) return;
    uint32_t acc = 0;
    for (uint32_t d = lane; d < nb; d += 64)
        acc += COLUMN ? in[static_cast<size_t>(d) * ntiles + tile] : in[static_cast<size_t>(tile) * nb + d];
    if (acc == 0xdeadbeefu) atomicAdd(sink, 1ull);
}

struct Timer {
    hipEvent_t a, b;
    Timer() {
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
    }
    void start() { CK(hipEventRecord(a)); }
    float stop() {
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    }
};

template <typename F>
void bench(const char* name, double bytes, F launch, int reps = 10) {
    Timer t;
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps; r++) {
        t.start();
        launch();
        const float ms = t.stop();
        best = ms < best ? ms : best;
        sum += ms;
    }
    printf("{\"kernel\": \"%s\", \"avg_ms\": %.4f, \"best_ms\": %.4f, \"GBps_avg\": %.1f, \"GBps_best\": %.1f}\n", name,
           sum / reps, best, bytes / (sum / reps) / 1e6, bytes / best / 1e6);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 200000000ull;  // tuples
    longlong2 *in, *out;
    long long* op;
    unsigned long long* sink;
    CK(hipMalloc(&in, n * 16));
    CK(hipMalloc(&out, n * 16));
    CK(hipMalloc(&op, n * 8));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(in, 1, n * 16));
    CK(hipMemset(out, 0, n * 16));
    const double B = n * 16.0;
#define GRID(T) dim3((n + (T)-1) / (T))
    bench("copy16 b256 i4", 2 * B, [&] { k_copy16<256, 4, false><<<GRID(1024), 256>>>(in, out, n); });
    bench("copy16 b256 i8", 2 * B, [&] { k_copy16<256, 8, false><<<GRID(2048), 256>>>(in, out, n); });
    bench("copy16 b256 i16", 2 * B, [&] { k_copy16<256, 16, false><<<GRID(4096), 256>>>(in, out, n); });
    bench("copy16 b512 i8", 2 * B, [&] { k_copy16<512, 8, false><<<GRID(4096), 512>>>(in, out, n); });
    bench("copy16_nt b256 i8", 2 * B, [&] { k_copy16<256, 8, true><<<GRID(2048), 256>>>(in, out, n); });
    bench("copy16_nt b256 i16", 2 * B, [&] { k_copy16<256, 16, true><<<GRID(4096), 256>>>(in, out, n); });
    bench("read16 b256 i8", B, [&] { k_read16<256, 8><<<GRID(2048), 256>>>(in, sink, n); });
    bench("read16 b256 i16", B, [&] { k_read16<256, 16><<<GRID(4096), 256>>>(in, sink, n); });
    bench("write16 b256 i8", B, [&] { k_write16<256, 8, false><<<GRID(2048), 256>>>(out, n); });
    bench("write16_nt b256 i8", B, [&] { k_write16<256, 8, true><<<GRID(2048), 256>>>(out, n); });
    const size_t nt = (n / 4096) * 4096;
    const double Bt = nt * 32.0;
    long long* ok = reinterpret_cast<long long*>(out);
    if (argc > 2) for (int R : {16, 64, 256}) {
        char name[64];
        snprintf(name, sizeof name, "runs_soa R%d", R);
        bench(name, Bt, [&] { k_runs<256, 16, false, false, false><<<nt / 4096, 256>>>(in, ok, op, nt, R); });
        snprintf(name, sizeof name, "runs_soa_remap R%d", R);
        bench(name, Bt, [&] { k_runs<256, 16, false, false, true><<<nt / 4096, 256>>>(in, ok, op, nt, R); });
        snprintf(name, sizeof name, "runs_soa_remap_nt R%d", R);
        bench(name, Bt, [&] { k_runs<256, 16, false, true, true><<<nt / 4096, 256>>>(in, ok, op, nt, R); });
        snprintf(name, sizeof name, "runs_aos_remap R%d", R);
        bench(name, Bt, [&] { k_runs<256, 16, true, false, true><<<nt / 4096, 256>>>(in, ok, op, nt, R); });
        snprintf(name, sizeof name, "runs_aos_remap_nt R%d", R);
        bench(name, Bt, [&] { k_runs<256, 16, true, true, true><<<nt / 4096, 256>>>(in, ok, op, nt, R); });
    }
    {
        const uint32_t ntiles = 48832, nb = 256;
        uint32_t* h = reinterpret_cast<uint32_t*>(op);
        const double hb = 4.0 * ntiles * nb;
        const dim3 g((ntiles / 4 + 7) & ~7u);
        bench("histw column", hb, [&] { k_histw<true, false><<<g, 256>>>(h, ntiles, nb); });
        bench("histw column remap", hb, [&] { k_histw<true, true><<<g, 256>>>(h, ntiles, nb); });
        bench("histw row", hb, [&] { k_histw<false, false><<<g, 256>>>(h, ntiles, nb); });
        bench("histw row remap", hb, [&] { k_histw<false, true><<<g, 256>>>(h, ntiles, nb); });
        bench("histr column remap", hb, [&] { k_histr<true, true><<<g, 256>>>(h, ntiles, nb, sink); });
        bench("histr row remap", hb, [&] { k_histr<false, true><<<g, 256>>>(h, ntiles, nb, sink); });
    }
    return 0;
}
