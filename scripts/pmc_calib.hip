// Calibration of rocprofv3's memory-side counters (FETCH_SIZE, TCC_EA0_RDREQ,
// TCC_HIT/MISS) for the access widths the join's kernels use, on a known byte
// count. MI355X_MICROARCH.md calibrates FETCH_SIZE only for 16-B-per-lane
// streaming reads (reported at exactly half); the counting probe reads 8-B hash
// codes per lane and random 16-B home slots, so each pattern gets its own
// known-answer kernel here.
//   hipcc --offload-arch=gfx950 -O3 -o gpurun_out/pmc_calib scripts/pmc_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -- gpurun_out/pmc_calib
// Every kernel reads exactly `bytes` (printed) once; names say the pattern.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));       \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// 8 B per lane, coalesced (a wave reads 512 contiguous bytes)
__global__ __launch_bounds__(256) void k_read8(const long long* __restrict__ in, size_t n, unsigned long long* sink) {
    long long acc = 0;
    for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256)
        acc ^= in[i];
    if (acc == 0x7fffffffffffffffll) atomicAdd(sink, 1ull);
}

// 16 B per lane, coalesced (the guide's calibrated case)
__global__ __launch_bounds__(256) void k_read16(const longlong2* __restrict__ in, size_t n, unsigned long long* sink) {
    long long acc = 0;
    for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) {
        const longlong2 v = in[i];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x7fffffffffffffffll) atomicAdd(sink, 1ull);
}

// 8 B of every 16-B tuple (the key of an AoS tuple: the pass-1 load pattern)
__global__ __launch_bounds__(256) void k_read8of16(const longlong2* __restrict__ in, size_t n, unsigned long long* sink) {
    long long acc = 0;
    for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256)
        acc ^= in[i].x;
    if (acc == 0x7fffffffffffffffll) atomicAdd(sink, 1ull);
}

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// random 16-B reads over a region of `slots` 16-B slots (one per lane)
__global__ __launch_bounds__(256) void k_rand16(const longlong2* __restrict__ in, size_t slots, size_t nreads,
                                                unsigned long long* sink) {
    long long acc = 0;
    for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < nreads; i += static_cast<size_t>(gridDim.x) * 256) {
        const longlong2 v = in[mix(i) % slots];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x7fffffffffffffffll) atomicAdd(sink, 1ull);
}

// 8 B per lane coalesced writes
__global__ __launch_bounds__(256) void k_write8(long long* __restrict__ out, size_t n) {
    for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256)
        out[i] = static_cast<long long>(i);
}

int main() {
    const size_t n16 = 200000000ull;   // 3.2 GB of 16-B tuples
    longlong2* buf;
    unsigned long long* sink;
    CK(hipMalloc(&buf, n16 * 16));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(buf, 1, n16 * 16));
    const dim3 g(256 * 8), b(256);
    // 1.6 GB of 8-B codes (the probe's stream)
    k_read8<<<g, b>>>(reinterpret_cast<const long long*>(buf), n16, sink);
    printf("k_read8 bytes %zu\n", n16 * 8);
    k_read16<<<g, b>>>(buf, n16, sink);
    printf("k_read16 bytes %zu\n", n16 * 16);
    k_read8of16<<<g, b>>>(buf, n16, sink);
    printf("k_read8of16 bytes(lines) %zu\n", n16 * 16);
    // 100M random 16-B reads in 1 MB (L2-resident) and in 2 GB (memory)
    k_rand16<<<g, b>>>(buf, (1u << 20) / 16, 100000000ull, sink);
    printf("k_rand16 L2 reads %llu\n", 100000000ull);
    k_rand16<<<g, b>>>(buf, (2ull << 30) / 16, 100000000ull, sink);
    printf("k_rand16 HBM reads %llu\n", 100000000ull);
    k_write8<<<g, b>>>(reinterpret_cast<long long*>(buf), n16);
    printf("k_write8 bytes %zu\n", n16 * 8);
    CK(hipDeviceSynchronize());
    CK(hipFree(buf));
    return 0;
}
