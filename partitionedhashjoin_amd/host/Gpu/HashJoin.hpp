// Drop-in GPU joiners with the reference's HashJoiner API:
//
//   RadixClustering::HashJoiner<HashTableFactory, HasherType>(Configuration, pool, hasher, factory)
//     .Run(tableA /*build*/, tableB /*probe*/, timer)       src/RadixCluster/HashJoin.hpp:92-135, 190-241
//   NoPartitioning::HashJoiner<HashTableFactory>(Configuration, pool, factory)
//     .Run(tableA, tableB, timer)                           src/NoPartitioning/HashJoin.hpp:15-41, 54-187
//
// The thread-pool slot of the reference constructors takes a Gpu::Device (one
// phj_ctx: device, stream, workspace). Run() hands &(*table)[0] / GetSize()
// to the C ABI (include/phj.h), runs partition / build / probe on the MI355X,
// drives the timer with the device-measured phase times and, like the
// reference, returns an empty Table<JoinedTuple> (counts only) unless
// GpuConfiguration::Materialize asks for the rows (phj_join_materialize:
// one JoinedTuple per matching probe tuple, copied back); the matched
// count is logged ("Joined N tuples", RadixCluster/HashJoin.hpp:320-321),
// added to the results as `matches`, and kept in GetNumberOfJoinedTuples().
// C ABI errors surface as std::runtime_error / std::invalid_argument, which the
// CLI catches and turns into exit(1) (src/main.cpp:277-281).
#pragma once

#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "Common/Configuration.hpp"
#include "Common/Hashers.hpp"
#include "Common/Logger.hpp"
#include "Common/Results.hpp"
#include "Common/Table.hpp"
#include "phj.h"

namespace Gpu {

// One phj_ctx: one HIP device, or several (the multi-GPU join: the relations
// are range-sharded across them, RCCL exchanges the partitioned build keys).
// The reference's thread pool (src/main.cpp:235-241) sits in this slot.
class Device {
   public:
    explicit Device(int device = 0) {
        const int rc = phj_ctx_create_device(device, &m_ctx);
        if (rc != PHJ_OK) throw std::runtime_error("phj_ctx_create_device(" + std::to_string(device) + ") failed");
    }
    Device(const std::vector<int>& devices, uint32_t flags) {
        const int rc = phj_ctx_create_ex(static_cast<int>(devices.size()), devices.data(), flags, &m_ctx);
        if (rc != PHJ_OK)
            throw std::runtime_error("phj_ctx_create_ex(" + std::to_string(devices.size()) + " devices) failed");
        m_gpus = static_cast<int>(devices.size());
    }
    int NumberOfGpus() const { return m_gpus; }
    ~Device() { phj_ctx_destroy(m_ctx); }
    Device(const Device&) = delete;
    Device& operator=(const Device&) = delete;

    phj_ctx* Get() const { return m_ctx; }

    void Check(int rc) const {
        if (rc == PHJ_OK) return;
        const std::string msg = phj_last_error(m_ctx);
        if (rc == PHJ_ERR_INVALID) throw std::invalid_argument(msg);
        throw std::runtime_error(msg);
    }

    void Upload(int side, const Common::Table<Common::Tuple>& t) {
        Check(phj_relation_upload(m_ctx, side, reinterpret_cast<const phj_tuple*>(t.Data()), t.GetSize()));
    }

   private:
    phj_ctx* m_ctx = nullptr;
    int m_gpus = 1;
};

namespace internal {

inline std::chrono::nanoseconds ms_to_ns(double ms) {
    return std::chrono::nanoseconds(static_cast<int64_t>(std::llround(ms * 1e6)));
}

// phj_join or, with rows requested, phj_join_materialize + the rows copied
// into the returned table
inline std::shared_ptr<Common::Table<Common::JoinedTuple>> join(Device& dev, const phj_join_params& p,
                                                                phj_join_result& r, bool materialize) {
    if (!materialize) {
        dev.Check(phj_join(dev.Get(), &p, &r));
        return std::make_shared<Common::Table<Common::JoinedTuple>>(Common::generate_uuid());
    }
    static_assert(sizeof(Common::JoinedTuple) == sizeof(phj_joined), "JoinedTuple layout");
    dev.Check(phj_join_materialize(dev.Get(), &p, &r));
    auto out = std::make_shared<Common::Table<Common::JoinedTuple>>(r.matches, Common::generate_uuid());
    dev.Check(phj_joined_download(dev.Get(), reinterpret_cast<phj_joined*>(out->Data()), r.matches));
    return out;
}

inline void add_device_results(Common::IHashJoinTimer& timer, const phj_join_result& r, int gpus) {
    timer.AddResult("matches", std::to_string(r.matches));
    timer.AddResult("gpus", std::to_string(gpus));
    timer.AddResult("exchange_us", std::to_string(static_cast<int64_t>(std::llround(r.exchange_ms * 1e3))));
    timer.AddResult("device_total_us", std::to_string(static_cast<int64_t>(std::llround(r.total_ms * 1e3))));
    timer.AddResult("algorithmic_bytes", std::to_string(r.algorithmic_bytes));
}

}  // namespace internal

namespace RadixClustering {

template <typename HashTableFactory, typename HasherType>
class HashJoiner {
   public:
    HashJoiner(::RadixClustering::Configuration configuration, std::shared_ptr<Device> device,
               const HasherType& hasher, const HashTableFactory& hashTableFactory,
               const Common::GpuConfiguration& gpu = Common::GpuConfiguration{})
        : m_configuration(configuration),
          m_device(std::move(device)),
          m_hasher(hasher),
          m_factory(hashTableFactory),
          m_gpu(gpu),
          m_logger(Common::GetNewLogger()) {
        Common::AddComponentAttributeToLogger(m_logger, "RadixPartitioning.HashJoiner");
    }

    // tableA is the build relation, tableB the probe relation (HashJoin.hpp:99)
    std::shared_ptr<Common::Table<Common::JoinedTuple>> Run(
        std::shared_ptr<Common::Table<Common::Tuple>> tableA, std::shared_ptr<Common::Table<Common::Tuple>> tableB,
        std::shared_ptr<Common::IHashJoinTimer> timer = std::make_shared<Common::NoOpHashJoinTimer>()) {
        m_device->Upload(PHJ_SIDE_BUILD, *tableA);
        m_device->Upload(PHJ_SIDE_PROBE, *tableB);
        return RunResident(timer);
    }

    // Join the relations already resident on the device (uploaded or generated there).
    std::shared_ptr<Common::Table<Common::JoinedTuple>> RunResident(
        std::shared_ptr<Common::IHashJoinTimer> timer = std::make_shared<Common::NoOpHashJoinTimer>()) {
        phj_join_params p{};
        p.algo = PHJ_ALGO_RADIX;
        p.hash = HasherType::kKind;
        p.hash_seed = m_hasher.Seed();
        p.flags = HashTableFactory::kTableFlags;   // the factory's table kind
        if (m_gpu.RadixBits[0] > 0) {
            p.num_partitions = 0;
            p.radix_bits[0] = static_cast<uint8_t>(m_gpu.RadixBits[0]);
            p.radix_bits[1] = static_cast<uint8_t>(m_gpu.RadixBits[1]);
        } else {
            if (m_configuration.NumberOfPartitions == 0 || m_configuration.NumberOfPartitions > 0xffffffffull)
                throw std::invalid_argument("number of partitions must be in [1, 2^32)");
            p.num_partitions = static_cast<uint32_t>(m_configuration.NumberOfPartitions);
        }
        LOG(m_logger, Common::debug) << "Starting hash partitioning.";
        phj_join_result r;
        std::memset(&r, 0, sizeof(r));
        // workspace allocation stays outside the timed phases, as the reference's
        // partitioned-table allocation does (RadixCluster/HashJoin.hpp:195-198)
        m_device->Check(phj_prepare(m_device->Get(), &p));
        auto joined = internal::join(*m_device, p, r, m_gpu.Materialize);
        // partition: wall of both partition pipelines; build / probe: device phases
        timer->SetPartitionPhaseDuration(internal::ms_to_ns(r.partition_ms));
        timer->SetBuildPhaseDuration(internal::ms_to_ns(r.build_ms));
        timer->SetProbePhaseDuration(internal::ms_to_ns(r.probe_ms));
        internal::add_device_results(*timer, r, m_device->NumberOfGpus());
        timer->AddResult("partitions", std::to_string(r.num_partitions));
        m_joined = r.matches;
        m_last = r;
        LOG(m_logger, Common::debug) << "Joined  " << r.matches << " tuples";
        LOG(m_logger, Common::debug) << "Finished hash partitioning.";
        return joined;
    }

    uint64_t GetNumberOfJoinedTuples() const { return m_joined; }
    const phj_join_result& GetLastResult() const { return m_last; }

   private:
    ::RadixClustering::Configuration m_configuration;
    std::shared_ptr<Device> m_device;
    HasherType m_hasher;
    HashTableFactory m_factory;
    Common::GpuConfiguration m_gpu;
    Common::LoggerType m_logger;
    uint64_t m_joined = 0;
    phj_join_result m_last{};
};

}  // namespace RadixClustering

namespace NoPartitioning {

template <typename HashTableFactory>
class HashJoiner {
   public:
    HashJoiner(::NoPartitioning::Configuration configuration, std::shared_ptr<Device> device,
               const HashTableFactory& hashTableFactory, const Common::GpuConfiguration& gpu = Common::GpuConfiguration{})
        : m_configuration(configuration),
          m_device(std::move(device)),
          m_factory(hashTableFactory),
          m_gpu(gpu),
          m_logger(Common::GetNewLogger()) {
        Common::AddComponentAttributeToLogger(m_logger, "NoPartitioning.HashJoiner");
    }

    std::shared_ptr<Common::Table<Common::JoinedTuple>> Run(
        std::shared_ptr<Common::Table<Common::Tuple>> tableA, std::shared_ptr<Common::Table<Common::Tuple>> tableB,
        std::shared_ptr<Common::IHashJoinTimer> timer = std::make_shared<Common::NoOpHashJoinTimer>()) {
        m_device->Upload(PHJ_SIDE_BUILD, *tableA);
        m_device->Upload(PHJ_SIDE_PROBE, *tableB);
        return RunResident(timer);
    }

    std::shared_ptr<Common::Table<Common::JoinedTuple>> RunResident(
        std::shared_ptr<Common::IHashJoinTimer> timer = std::make_shared<Common::NoOpHashJoinTimer>()) {
        using Hasher = typename HashTableFactory::Hasher;
        phj_join_params p{};
        p.algo = PHJ_ALGO_NO_PARTITIONING;
        p.hash = Hasher::kKind;
        p.hash_seed = m_factory.GetHasher().Seed();
        p.table_ratio = m_gpu.TableRatio;
        LOG(m_logger, Common::debug) << "Starting hash partitioning.";
        phj_join_result r;
        std::memset(&r, 0, sizeof(r));
        // workspace allocation stays outside the timed phases, as the reference's
        // partitioned-table allocation does (RadixCluster/HashJoin.hpp:195-198)
        m_device->Check(phj_prepare(m_device->Get(), &p));
        auto joined = internal::join(*m_device, p, r, m_gpu.Materialize);
        timer->SetBuildPhaseDuration(internal::ms_to_ns(r.build_ms));
        // the reference's probe figure runs from the build start (Results.hpp:202)
        timer->SetProbePhaseDuration(internal::ms_to_ns(r.build_ms + r.probe_ms));
        timer->SetPartitionPhaseDuration(std::chrono::nanoseconds(0));
        internal::add_device_results(*timer, r, m_device->NumberOfGpus());
        timer->AddResult("probe_only_us", std::to_string(static_cast<int64_t>(std::llround(r.probe_ms * 1e3))));
        m_joined = r.matches;
        m_last = r;
        LOG(m_logger, Common::debug) << "Joined " << r.matches << " tuples.";
        LOG(m_logger, Common::debug) << "Finished hash partitioning.";
        return joined;
    }

    uint64_t GetNumberOfJoinedTuples() const { return m_joined; }
    const phj_join_result& GetLastResult() const { return m_last; }

   private:
    ::NoPartitioning::Configuration m_configuration;
    std::shared_ptr<Device> m_device;
    HashTableFactory m_factory;
    Common::GpuConfiguration m_gpu;
    Common::LoggerType m_logger;
    uint64_t m_joined = 0;
    phj_join_result m_last{};
};

}  // namespace NoPartitioning
}  // namespace Gpu
