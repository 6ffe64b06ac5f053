// Host check of csrc/phj_pow.h against this machine's glibc pow (tests/test_pow.py).
// Prints "<variant> <mismatches> <total>" for the FMA and the non-FMA restatement.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "phj_pow.h"

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    uint64_t bad[2] = {0, 0}, total = 0;
    auto check = [&](double x, double y) {
        const double ref = std::pow(x, y);
        const double a = phj::glibc_pow::pow<true>(x, y), b = phj::glibc_pow::pow<false>(x, y);
        uint64_t ur, ua, ub;
        std::memcpy(&ur, &ref, 8);
        std::memcpy(&ua, &a, 8);
        std::memcpy(&ub, &b, 8);
        bad[0] += ua != ur;
        bad[1] += ub != ur;
        if (ua != ur && bad[0] <= 25) std::fprintf(stderr, "fma mismatch pow(%a, %a) = %a vs %a\n", x, y, ref, a);
        total++;
    };
    const double alphas[] = {1.05, 1.25, 0.99, 1.5, 2.0, 0.5, 1.1};
    for (uint64_t i = 0; i < n; i++) {
        // the generator's calls (Zipf.cpp:29-50): card^skew, (u*norm*skew + alpha)^(1/skew),
        // sample^-alpha, inv^-alpha, skew = 1.001 - alpha (or the +-0.01 clamp)
        const double alpha = alphas[i % 7];
        double skew = 1.001 - alpha;
        if (std::fabs(1.0 - alpha) < 0.01) skew = 0.01 * ((1.0 - alpha < 0) ? 1 : -1);
        const double card = std::floor(1.0 + U(rng) * 2e8);
        const double norm = (std::pow(card, skew) - alpha) / skew;
        check(card, skew);
        const double u = U(rng);
        const double base = (u * norm) * skew + alpha;
        if (base > 0) check(base, 1.0 / skew);
        const double inv = std::pow(base, 1.0 / skew);
        check(std::floor(inv + 1), -alpha);
        if (inv > 0) check(inv, -alpha);
        // random finite positive x and moderate y
        const double x = std::ldexp(1.0 + U(rng), static_cast<int>(rng() % 2000) - 1000);
        const double y = (U(rng) - 0.5) * std::ldexp(1.0, static_cast<int>(rng() % 20) - 10);
        if (y != 0 && std::isfinite(std::pow(x, y)) && std::pow(x, y) > 0x1p-1000) check(x, y);
    }
    std::printf("fma %llu %llu\nnofma %llu %llu\n", (unsigned long long)bad[0], (unsigned long long)total,
                (unsigned long long)bad[1], (unsigned long long)total);
    return 0;
}
