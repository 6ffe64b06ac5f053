// Relation generators of the reference (src/DataGenerator/{Sequential,Zipf},
// src/Common/Random) on host threads, with an explicit seed: batch b of
// kGenBatch tuples draws from its own Park-Miller LCG stream seeded
// 1 + ((seed mod M) * 1000003 + b) mod M, M = 2^31 - 2 (the reference seeds
// each worker batch from std::random_device, Zipf.cpp:86, so its tables are
// not reproducible). The device generator (phj_relation_generate_*) uses the
// same streams, so shards and devices agree on the table definition.
#pragma once

#include <cstdint>
#include <memory>
#include <utility>

#include "Common/Table.hpp"

namespace Common {

// MultiplicativeLCGRandomNumberGenerator (src/Common/Random.cpp:9-30)
class MultiplicativeLCGRandomNumberGenerator {
   public:
    explicit MultiplicativeLCGRandomNumberGenerator(long seed) : m_state(seed) {}
    double Next();

   private:
    long m_state;
};

long BatchSeed(uint64_t baseSeed, uint64_t batch);

}  // namespace Common

namespace DataGenerator {

constexpr uint64_t kGenBatch = 4096;

class Sequential {
   public:
    struct Parameters {
        int64_t start;
        size_t threads = 0;  // 0: hardware_concurrency() - 1
    };
    static void FillTable(std::shared_ptr<Common::Table<Common::Tuple>> table, const Parameters& parameters);
};

class Zipf {
   public:
    struct Parameters {
        double alpha;
        std::pair<int64_t, int64_t> range;  // closed [lo, hi]
        uint64_t seed;
        size_t threads = 0;
    };
    // throws std::invalid_argument like Zipf.cpp:19-21,61-67
    static void FillTable(std::shared_ptr<Common::Table<Common::Tuple>> table, const Parameters& parameters);
    // Zipf::generate (Zipf.cpp:14-56)
    static uint64_t Generate(double alpha, uint64_t cardinality, Common::MultiplicativeLCGRandomNumberGenerator& g);
};

}  // namespace DataGenerator
