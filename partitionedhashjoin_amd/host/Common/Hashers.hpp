// Hashers of the reference API (src/Common/XXHasher.hpp:9-26, IHasher.hpp):
// Hash(key, cardinality) = hash % cardinality. XXHasher draws a random seed
// like the reference unless one is given; Murmur3Hasher is the BASELINE C2
// option. On the device the same functions run per lane (csrc/phj_hash.h);
// here they are host evaluations of that same header, for API parity.
#pragma once

#include <cstdint>
#include <limits>
#include <random>

#include "phj.h"
#include "phj_hash.h"

namespace Common {

class IHasher {
   public:
    virtual uint64_t Hash(int64_t key, size_t cardinality) = 0;
    virtual ~IHasher() = default;
};

namespace internal {
inline uint64_t random_seed() {
    std::random_device rd;
    std::mt19937 gen(rd());
    std::uniform_int_distribution<uint64_t> dist(0, std::numeric_limits<uint64_t>::max());
    return dist(gen);
}
}  // namespace internal

class XXHasher : public IHasher {
   public:
    static constexpr int kKind = PHJ_HASH_XXH3;
    XXHasher() : m_seed(internal::random_seed()) {}
    explicit XXHasher(uint64_t seed) : m_seed(seed) {}
    uint64_t Hash(int64_t key, size_t cardinality) override {
        return phj::xxh3_8(static_cast<uint64_t>(key), m_seed) % cardinality;
    }
    uint64_t Seed() const { return m_seed; }

   private:
    uint64_t m_seed;
};

class Murmur3Hasher : public IHasher {
   public:
    static constexpr int kKind = PHJ_HASH_MURMUR3;
    Murmur3Hasher() : m_seed(internal::random_seed()) {}
    explicit Murmur3Hasher(uint64_t seed) : m_seed(seed) {}
    uint64_t Hash(int64_t key, size_t cardinality) override {
        return phj::murmur3_fmix64(static_cast<uint64_t>(key), m_seed) % cardinality;
    }
    uint64_t Seed() const { return m_seed; }

   private:
    uint64_t m_seed;
};

}  // namespace Common

namespace HashTables {

// Table descriptors of the reference's factories (LinearProbing.hpp:16-18,
// 212-227; SeparateChaining.hpp:16-18, 279-294). The factory contributes its
// hasher, its size ratio (slots per build tuple = ratio x bucket slots) and
// the radix join's table kind: open-addressed code tables for LinearProbing,
// bucket-chained tables (PHJ_TABLE_CHAINED) for SeparateChaining. The
// no-partitioning join always uses its own global table.
struct LinearProbingConfiguration {
    double HASH_TABLE_SIZE_RATIO = 1.25;
};
struct SeparateChainingConfiguration {
    double HASH_TABLE_SIZE_RATIO = 0.25;
};

template <typename BucketValueType, size_t BucketSize, typename HasherType>
class LinearProbingFactory {
   public:
    using Hasher = HasherType;
    static constexpr uint8_t kTableFlags = 0;
    LinearProbingFactory(const LinearProbingConfiguration& configuration, HasherType hasher)
        : m_hasher(hasher), m_configuration(configuration) {}
    const HasherType& GetHasher() const { return m_hasher; }
    double SlotsPerTuple() const { return m_configuration.HASH_TABLE_SIZE_RATIO * BucketSize; }

   private:
    HasherType m_hasher;
    LinearProbingConfiguration m_configuration;
};

template <typename BucketValueType, size_t BucketSize, typename HasherType>
class SeparateChainingFactory {
   public:
    using Hasher = HasherType;
    static constexpr uint8_t kTableFlags = PHJ_TABLE_CHAINED;
    SeparateChainingFactory(const SeparateChainingConfiguration& configuration, HasherType hasher)
        : m_hasher(hasher), m_configuration(configuration) {}
    const HasherType& GetHasher() const { return m_hasher; }
    // heads x slots plus the overflow allocator's ceil(n/3) buckets (SeparateChaining.hpp:168-171)
    double SlotsPerTuple() const { return m_configuration.HASH_TABLE_SIZE_RATIO * BucketSize + 1.0; }

   private:
    HasherType m_hasher;
    SeparateChainingConfiguration m_configuration;
};

}  // namespace HashTables
