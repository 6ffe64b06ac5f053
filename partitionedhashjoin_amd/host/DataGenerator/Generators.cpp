#include "DataGenerator/Generators.hpp"

#include <algorithm>
#include <cmath>
#include <sstream>
#include <stdexcept>
#include <thread>
#include <vector>

namespace Common {

double MultiplicativeLCGRandomNumberGenerator::Next() {
    const long a = 16807, m = 2147483647, q = 127773, r = 2836;
    const long x_new = a * (m_state % q) - r * (m_state / q);
    m_state = x_new > 0 ? x_new : x_new + m;
    return static_cast<double>(m_state) / static_cast<double>(m);
}

long BatchSeed(uint64_t baseSeed, uint64_t batch) {
    const uint64_t M = 2147483646ULL;
    return static_cast<long>(1 + (((baseSeed % M) * 1000003ULL + batch) % M));
}

}  // namespace Common

namespace DataGenerator {

namespace {
size_t worker_count(size_t requested) {
    if (requested) return requested;
    const unsigned hc = std::thread::hardware_concurrency();
    return hc > 1 ? hc - 1 : 1;
}

template <typename F>
void parallel_batches(uint64_t n, size_t threads, F&& body) {
    const uint64_t batches = (n + kGenBatch - 1) / kGenBatch;
    const size_t w = std::max<size_t>(1, std::min<uint64_t>(threads, batches));
    std::vector<std::thread> pool;
    for (size_t t = 0; t < w; t++)
        pool.emplace_back([&, t] {
            for (uint64_t b = t; b < batches; b += w) body(b, b * kGenBatch, std::min(n, (b + 1) * kGenBatch));
        });
    for (auto& th : pool) th.join();
}
}  // namespace

void Sequential::FillTable(std::shared_ptr<Common::Table<Common::Tuple>> table, const Parameters& p) {
    const uint64_t n = table->GetSize();
    parallel_batches(n, worker_count(p.threads), [&](uint64_t, uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; i++) {
            (*table)[i].id = p.start + static_cast<int64_t>(i);
            (*table)[i].payload = static_cast<int64_t>(i);
        }
    });
}

uint64_t Zipf::Generate(double alpha, uint64_t cardinality, Common::MultiplicativeLCGRandomNumberGenerator& g) {
    constexpr double errorDifferential = 0.01;
    if (alpha < 0.01) throw std::invalid_argument("Skew parameter must be greater than 0.01.");
    double skew = 1.001 - alpha;
    if (const double diff = 1.0 - alpha; std::abs(diff) < errorDifferential) {
        skew = errorDifferential * ((diff < 0) ? 1 : -1);
        alpha = 1.0 - skew;
    }
    const double norm = (std::pow(static_cast<double>(cardinality), skew) - alpha) / skew;
    while (true) {
        const double u1 = g.Next();
        const double u2 = g.Next();
        double inv;
        if (u1 * norm <= 1.0) inv = u1 * norm;
        else inv = std::pow((u1 * norm) * skew + alpha, 1.0 / skew);
        const double sample = std::floor(inv + 1);
        const double densityOriginal = std::pow(sample, -alpha);
        const double densitySampling = sample <= 1.0 ? 1.0 / norm : std::pow(inv, -alpha) / norm;
        if (u2 < densityOriginal / (densitySampling * norm)) return static_cast<uint64_t>(sample);
    }
}

void Zipf::FillTable(std::shared_ptr<Common::Table<Common::Tuple>> table, const Parameters& p) {
    if (p.range.first >= p.range.second) {
        std::ostringstream msg;
        msg << "Range for Zipf generation is incorrectly specified: [" << p.range.first << ", " << p.range.second
            << "].";
        throw std::invalid_argument(msg.str());
    }
    if (p.alpha < 0.01) throw std::invalid_argument("Skew parameter must be greater than 0.01.");
    const uint64_t cardinality = static_cast<uint64_t>(p.range.second - p.range.first + 1);
    const int64_t correction = p.range.first - 1;
    const uint64_t n = table->GetSize();
    parallel_batches(n, worker_count(p.threads), [&](uint64_t b, uint64_t lo, uint64_t hi) {
        Common::MultiplicativeLCGRandomNumberGenerator g(Common::BatchSeed(p.seed, b));
        for (uint64_t i = lo; i < hi; i++) {
            (*table)[i].id = static_cast<int64_t>(Generate(p.alpha, cardinality, g)) + correction;
            (*table)[i].payload = static_cast<int64_t>(i);
        }
    });
}

}  // namespace DataGenerator
