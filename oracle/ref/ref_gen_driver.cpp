// ref_gen_driver.cpp — TEST INFRASTRUCTURE ONLY.
//
// Harness that links the reference's OWN, unmodified data-generator sources
// (/root/reference/src/Common/Random.cpp, DataGenerator/Zipf.cpp,
// DataGenerator/Sequential.cpp, Common/IThreadPool.cpp — compiled in place by
// oracle/ref/Makefile, never copied) and exposes them through a C ABI so
// tests/golden/make_golden.py can record golden vectors that pin the oracle's
// restatement. Only the harness-side pieces below are ours: a synchronous
// IThreadPool (the interface of src/Common/IThreadPool.hpp:36-49) and a seeded
// IRandomNumberGeneratorFactory (src/Common/Random.hpp:15-23) that hands out
// GetNewGenerator(seed_b) in batch order instead of std::random_device.
#include <cstdint>
#include <memory>
#include <vector>

#include "Common/IThreadPool.hpp"
#include "Common/Random.hpp"
#include "Common/Table.hpp"
#include "DataGenerator/Sequential.hpp"
#include "DataGenerator/Zipf.hpp"

namespace {

class SyncPool final : public Common::IThreadPool {
   public:
    explicit SyncPool(size_t workers) : m_workers(workers) {}
    std::future<Common::TasksErrorHolder> Push(std::function<void()>&& f) override {
        std::vector<std::function<void()>> v;
        v.push_back(std::move(f));
        return Push(std::move(v));
    }
    std::future<Common::TasksErrorHolder> Push(std::vector<std::function<void()>>&& fs) override {
        Common::TasksErrorHolder errors;
        for (auto& f : fs) {
            try {
                f();
            } catch (std::exception& e) {
                errors.Push(e);
            }
        }
        std::promise<Common::TasksErrorHolder> p;
        p.set_value(errors);
        return p.get_future();
    }
    std::future<Common::TasksErrorHolder> Push(std::shared_ptr<Common::IPipeline>) override {
        std::promise<Common::TasksErrorHolder> p;
        p.set_value(Common::TasksErrorHolder{});
        return p.get_future();
    }
    size_t GetNumberOfWorkers() const override { return m_workers; }
    void Stop() override {}

   private:
    size_t m_workers;
};

// Seeds batch b with 1 + ((base % M) * 1000003 + b) % M, M = 2^31 - 2
// (the oracle's or_batch_seed, phj_oracle.c).
class SeededFactory final : public Common::IRandomNumberGeneratorFactory {
   public:
    explicit SeededFactory(uint64_t base) : m_base(base), m_batch(0) {}
    std::shared_ptr<Common::IRandomNumberGenerator> GetNewGenerator() override {
        const uint64_t M = 2147483646ULL;
        long seed = static_cast<long>(1 + (((m_base % M) * 1000003ULL + m_batch++) % M));
        return m_inner.GetNewGenerator(seed);
    }
    std::shared_ptr<Common::IRandomNumberGenerator> GetNewGenerator(long seed) override {
        return m_inner.GetNewGenerator(seed);
    }

   private:
    uint64_t m_base;
    uint64_t m_batch;
    Common::MultiplicativeLCGRandomNumberGeneratorFactory m_inner;
};

// Exposes the protected Zipf::generate, exactly as tests/DataGenerator/ZipfTest.hpp:7-13 does.
class ZipfTester : public DataGenerator::Zipf {
   public:
    static uint64_t Gen(double alpha, uint64_t card,
                        std::shared_ptr<Common::IRandomNumberGenerator> g) {
        return DataGenerator::Zipf::generate(alpha, card, g);
    }
};

}  // namespace

extern "C" {

// n successive MultiplicativeLCGRandomNumberGenerator::Next() values from seed.
int ref_lcg_sequence(long seed, uint64_t n, double* out) {
    Common::MultiplicativeLCGRandomNumberGeneratorFactory f;
    auto g = f.GetNewGenerator(seed);
    for (uint64_t i = 0; i < n; i++) out[i] = g->Next();
    return 0;
}

// n successive Zipf::generate(alpha, card, LCG(seed)) samples; -1 on exception.
int ref_zipf_samples(double alpha, uint64_t card, long seed, uint64_t n, uint64_t* out) {
    try {
        Common::MultiplicativeLCGRandomNumberGeneratorFactory f;
        auto g = f.GetNewGenerator(seed);
        for (uint64_t i = 0; i < n; i++) out[i] = ZipfTester::Gen(alpha, card, g);
    } catch (std::exception&) {
        return -1;
    }
    return 0;
}

// Zipf::FillTable over [lo, hi] with n = batches * batch_size tuples, one
// worker per batch (so FillTable's batches are exactly the oracle's), seeded
// batch generators. out = 2*n int64 {id, payload}.
int ref_fill_zipf(double alpha, int64_t lo, int64_t hi, uint64_t base_seed, uint64_t batches,
                  uint64_t batch_size, int64_t* out) {
    const uint64_t n = batches * batch_size;
    auto pool = std::make_shared<SyncPool>(batches);
    auto table = std::make_shared<Common::Table<Common::Tuple>>(n, std::string("ref"));
    try {
        DataGenerator::Zipf::Parameters p{alpha,
                                          std::make_pair(static_cast<size_t>(lo),
                                                         static_cast<size_t>(hi)),
                                          std::make_shared<SeededFactory>(base_seed), batch_size};
        auto fut = DataGenerator::Zipf::FillTable(pool, table, p);
        auto errs = fut.get();
        if (!errs.Empty()) return -1;
    } catch (std::exception&) {
        return -1;
    }
    for (uint64_t i = 0; i < n; i++) {
        out[2 * i] = (*table)[i].id;
        out[2 * i + 1] = (*table)[i].payload;
    }
    return 0;
}

// Sequential::FillTable(start) over n tuples.
int ref_fill_sequential(int64_t start, uint64_t n, int64_t* out) {
    auto pool = std::make_shared<SyncPool>(4);
    auto table = std::make_shared<Common::Table<Common::Tuple>>(n, std::string("ref"));
    auto fut = DataGenerator::Sequential::FillTable(pool, table,
                                                    DataGenerator::Sequential::Parameters{start});
    auto errs = fut.get();
    if (!errs.Empty()) return -1;
    for (uint64_t i = 0; i < n; i++) {
        out[2 * i] = (*table)[i].id;
        out[2 * i + 1] = (*table)[i].payload;
    }
    return 0;
}
}
