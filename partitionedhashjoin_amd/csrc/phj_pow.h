// phj_pow.h — the pow() of the reference's Zipf generator, bit for bit, on the
// device.
//
// src/DataGenerator/Zipf.cpp:14-56 draws samples with std::pow, i.e. glibc's
// pow (>= 2.28: the log/exp algorithm of ARM's optimized-routines, < 0.52 ulp,
// not correctly rounded). The device libm pow rounds differently on ~1% of
// the generator's calls, and one differing rejection test shifts a batch's LCG
// stream. This restates glibc's evaluation over its own tables
// (phj_pow_tables.h, read from libm by scripts/gen_pow_tables.py) in the
// operation order of its FMA build: the x86-64 ifunc variant a Zen/Xeon host
// with FMA selects, compiled by GCC with the default -ffp-contract=fast, so
// besides the source's explicit fma() every product whose only use is an
// addition is fused (written out below as FMA(...); nothing else contracts).
// Checked against the host's pow on tens of millions of generator-domain and
// random arguments (tests/test_pow.py), and device samples against the host
// generator (tests/test_gpu_parity.py::test_gpu_generators).
//
// Attribution: the algorithm (log with a 128-entry table, exp with a 2^7
// table, their polynomials and the special-case handling) is that of ARM's
// optimized-routines math library (pow.c / pow_log_data.c / exp_data.c, MIT
// OR Apache-2.0 WITH LLVM-exception), as shipped in glibc >= 2.28
// (sysdeps/ieee754/dbl-64/e_pow.c, LGPL-2.1+). It is restated here from that
// published algorithm, not copied; the coefficient tables are read from the
// host's libm binary at generation time (phj_pow_tables.h).
#pragma once

#include <cstdint>
#include <cstring>

#include "phj_pow_tables.h"

#if defined(__HIPCC__)
#define PHJ_POW_HD __host__ __device__
#else
#define PHJ_POW_HD
#endif

namespace phj {
namespace glibc_pow {

PHJ_POW_HD inline uint64_t as_u64(double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}
PHJ_POW_HD inline double as_f64(uint64_t u) {
    double x;
    std::memcpy(&x, &u, 8);
    return x;
}
PHJ_POW_HD inline uint32_t top12(double x) { return static_cast<uint32_t>(as_u64(x) >> 52); }

// log(x) = hi + tail with ~15 extra bits (pow.c log_inline). ix: bits of x.
template <bool FMA>
PHJ_POW_HD inline double log_inline(uint64_t ix, double* tail) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    using namespace powtab;
    constexpr uint64_t OFF = 0x3fe6955500000000ull;
    const uint64_t tmp = ix - OFF;
    const int i = static_cast<int>((tmp >> (52 - 7)) % 128);
    const int k = static_cast<int>(static_cast<int64_t>(tmp) >> 52);
    const uint64_t iz = ix - (tmp & (0xfffull << 52));
    const double z = as_f64(iz);
    const double kd = static_cast<double>(k);
    const double invc = kLogTab[i][0], logc = kLogTab[i][1], logctail = kLogTab[i][2];
    double r, rhi = 0, rlo = 0;
    if constexpr (FMA) {
        r = __builtin_fma(z, invc, -1.0);
    } else {
        const double zhi = as_f64((iz + (1ull << 31)) & (~0ull << 32));
        const double zlo = z - zhi;
        rhi = zhi * invc - 1.0;
        rlo = zlo * invc;
        r = rhi + rlo;
    }
    const double t1 = FMA ? __builtin_fma(kd, kLn2hi, logc) : kd * kLn2hi + logc;
    const double t2 = t1 + r;
    const double lo1 = FMA ? __builtin_fma(kd, kLn2lo, logctail) : kd * kLn2lo + logctail;
    const double lo2 = t1 - t2 + r;
    const double* A = kLogPoly;
    const double ar = A[0] * r;
    const double ar2 = r * ar;
    const double ar3 = r * ar2;
    double hi, lo3, lo4;
    if constexpr (FMA) {
        hi = t2 + ar2;
        lo3 = __builtin_fma(ar, r, -ar2);
        lo4 = t2 - hi + ar2;
    } else {
        const double arhi = A[0] * rhi;
        const double arhi2 = rhi * arhi;
        hi = t2 + arhi2;
        lo3 = rlo * (ar + arhi);
        lo4 = t2 - hi + arhi2;
    }
    double lo;
    if constexpr (FMA) {
        // p = ar3 * (A1 + r A2 + ar2 (A3 + r A4 + ar2 (A5 + r A6))), fused into lo
        const double q5 = __builtin_fma(r, A[6], A[5]);
        const double q3 = __builtin_fma(ar2, q5, __builtin_fma(r, A[4], A[3]));
        const double q1 = __builtin_fma(ar2, q3, __builtin_fma(r, A[2], A[1]));
        lo = __builtin_fma(ar3, q1, lo1 + lo2 + lo3 + lo4);
    } else {
        const double p = ar3 * (A[1] + r * A[2] + ar2 * (A[3] + r * A[4] + ar2 * (A[5] + r * A[6])));
        lo = lo1 + lo2 + lo3 + lo4 + p;
    }
    const double y = hi + lo;
    *tail = hi - y + lo;
    return y;
}

// scale * (1 + tmp) when the exponent of scale over- or underflowed (pow.c specialcase)
template <bool FMA>
PHJ_POW_HD inline double exp_specialcase(double tmp, uint64_t sbits, uint64_t ki) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    if ((ki & 0x80000000ull) == 0) {
        sbits -= 1009ull << 52;
        const double scale = as_f64(sbits);
        return 0x1p1009 * (FMA ? __builtin_fma(scale, tmp, scale) : scale + scale * tmp);
    }
    // k < 0: scale * tmp also feeds the subnormal rounding below, a use in
    // another basic block, so GCC fuses neither addition here
    sbits += 1022ull << 52;
    const double scale = as_f64(sbits);
    double y = scale + scale * tmp;
    if ((y < 0 ? -y : y) < 1.0) {
        const double one = y < 0.0 ? -1.0 : 1.0;
        double lo = scale - y + scale * tmp;
        const double hi = one + y;
        lo = one - hi + y + lo;
        y = (hi + lo) - one;
        if (y == 0) y = as_f64(sbits & 0x8000000000000000ull);
    }
    return 0x1p-1022 * y;
}

// exp(x + xtail) (pow.c exp_inline, sign_bias 0: the generator's x is > 0)
template <bool FMA>
PHJ_POW_HD inline double exp_inline(double x, double xtail) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    using namespace powtab;
    uint32_t abstop = top12(x) & 0x7ff;
    if (abstop - top12(0x1p-54) >= top12(512.0) - top12(0x1p-54)) {
        if (abstop - top12(0x1p-54) >= 0x80000000u) return 1.0;
        if (abstop >= top12(1024.0)) return (as_u64(x) >> 63) ? 0.0 : __builtin_inf();
        abstop = 0;
    }
    double kd = FMA ? __builtin_fma(kInvLn2N, x, kShift) : kInvLn2N * x + kShift;
    const uint64_t ki = as_u64(kd);
    kd -= kShift;
    double r = FMA ? __builtin_fma(kd, kNegLn2loN, __builtin_fma(kd, kNegLn2hiN, x)) : x + kd * kNegLn2hiN + kd * kNegLn2loN;
    r += xtail;
    const uint64_t idx = 2 * (ki % 128);
    const uint64_t top = ki << (52 - 7);
    const double tail = as_f64(kExpTab[idx]);
    const uint64_t sbits = kExpTab[idx + 1] + top;
    const double r2 = r * r;
    double tmp;
    if constexpr (FMA) {
        const double b = __builtin_fma(r2, __builtin_fma(r, kExpPoly[1], kExpPoly[0]), tail + r);
        tmp = __builtin_fma(r2 * r2, __builtin_fma(r, kExpPoly[3], kExpPoly[2]), b);
    } else {
        tmp = tail + r + r2 * (kExpPoly[0] + r * kExpPoly[1]) + r2 * r2 * (kExpPoly[2] + r * kExpPoly[3]);
    }
    if (abstop == 0) return exp_specialcase<FMA>(tmp, sbits, ki);
    const double scale = as_f64(sbits);
    return FMA ? __builtin_fma(scale, tmp, scale) : scale + scale * tmp;
}

// pow(x, y) for finite x > 0 and finite y != 0 with 2^-65 <= |y| < 2^63:
// every call the Zipf generator makes. Other arguments return NaN (never
// produced by the generator; the caller's domain check keeps them out).
template <bool FMA = true>
PHJ_POW_HD inline double pow(double x, double y) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    uint64_t ix = as_u64(x);
    const uint64_t iy = as_u64(y);
    const uint32_t topx = top12(x), topy = top12(y);
    if (topx - 0x001 >= 0x7ff - 0x001 || (topy & 0x7ff) - 0x3be >= 0x43e - 0x3be) {
        if (x == 1.0) return 1.0;
        if (!(x > 0) || topx >= 0x7ff || (topy & 0x7ff) - 0x3be >= 0x43e - 0x3be) return __builtin_nan("");
        // subnormal x: normalise so the exponent becomes negative
        ix = as_u64(x * 0x1p52);
        ix &= 0x7fffffffffffffffull;
        ix -= 52ull << 52;
    }
    double lo;
    const double hi = log_inline<FMA>(ix, &lo);
    double ehi, elo;
    if constexpr (FMA) {
        ehi = y * hi;
        elo = __builtin_fma(y, lo, __builtin_fma(y, hi, -ehi));
    } else {
        const double yhi = as_f64(iy & (~0ull << 27));
        const double ylo = y - yhi;
        const double lhi = as_f64(as_u64(hi) & (~0ull << 27));
        const double llo = hi - lhi + lo;
        ehi = yhi * lhi;
        elo = ylo * lhi + y * llo;
    }
    return exp_inline<FMA>(ehi, elo);
}

}  // namespace glibc_pow
}  // namespace phj
