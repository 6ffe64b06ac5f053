// Configuration API of the reference (src/Common/Configuration.hpp:12-68,
// src/RadixCluster/Configuration.hpp, src/NoPartitioning/Configuration.hpp),
// plus additive device options (GpuConfiguration).
#pragma once

#include <cstdint>
#include <iostream>
#include <string>
#include <vector>

#include "Common/Logger.hpp"

namespace NoPartitioning {
struct Configuration {
    size_t MinBatchSize = 10000;
};
}  // namespace NoPartitioning

namespace RadixClustering {
struct Configuration {
    size_t MinBatchSize = 10000;
    size_t NumberOfPartitions = 32;
};
}  // namespace RadixClustering

namespace Common {

enum class JoinAlgorithmType : uint8_t {
    NoPartitioning = 0,
    RadixParitioning = 1,  // (sic) the reference's spelling
};
JoinAlgorithmType GetJoinAlgorithmTypeFromString(const std::string& algorithmType);
std::istream& operator>>(std::istream& in, JoinAlgorithmType& obj);
std::ostream& operator<<(std::ostream& os, JoinAlgorithmType algorithmType);

enum class ResultsFormat : uint8_t { JSON = 0 };
ResultsFormat GetResultsFormatFromString(const std::string& resultsFormat);
std::istream& operator>>(std::istream& in, ResultsFormat& obj);
std::ostream& operator<<(std::ostream& os, ResultsFormat resultsFormat);

enum class OutputType : uint8_t { File = 0 };
OutputType GetOutputTypeFromString(const std::string& outputType);
std::istream& operator>>(std::istream& in, OutputType& obj);
std::ostream& operator<<(std::ostream& os, OutputType outputType);

struct FileConfiguration {
    std::string Name;
};

struct OutputConfiguration {
    OutputType Type = OutputType::File;
    FileConfiguration File;
    void Validate() const;
};

struct ResultsFormatConfiguration {
    ResultsFormat Format = ResultsFormat::JSON;
    std::string TimeUnit = "ms";
    void Validate() const;
};

// Additive: where and how the join runs on the MI355X.
struct GpuConfiguration {
    int Device = 0;
    int Hash = 1;                    // PHJ_HASH_XXH3 = 0, PHJ_HASH_MURMUR3 = 1
    bool HashSet = false;            // --hash given (otherwise XXH3 for -p/no-partitioning)
    unsigned RadixBits[2] = {0, 0};  // --radix-bits b0,b1 (0,0: use NumberOfPartitions)
    bool HashSeedSet = false;
    uint64_t HashSeed = 0;
    uint64_t Seed = 20240601;        // data generator seed
    bool GenerateOnDevice = false;
    double TableRatio = 0.0;         // NoPartitioning slots per tuple (0: default)
    bool Materialize = false;        // --materialize on: Run() returns the joined rows (phj_join_materialize)
    std::vector<int> Devices;        // --gpus N / --devices a,b,..: the context's devices (empty: {Device})
    uint32_t ContextFlags = 0;       // --exchange rccl|local: PHJ_CTX_EXCHANGE / PHJ_CTX_LOCAL
};

struct Configuration {
    JoinAlgorithmType JoinType = JoinAlgorithmType::NoPartitioning;
    ResultsFormatConfiguration OutputFormatConfig;
    OutputConfiguration OutputConfig;

    size_t PrimaryRelationSize = 10'000'000;
    size_t SecondaryRelationSize = 200'000'000;
    double SkewParameter = 1.05;

    NoPartitioning::Configuration NoPartitioningConfig;
    RadixClustering::Configuration RadixClusteringConfig;

    LoggerConfiguration LoggerConfig;
    GpuConfiguration GpuConfig;
};

}  // namespace Common
