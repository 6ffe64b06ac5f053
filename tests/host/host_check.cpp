// Host-side checks of the C++ driver pieces that need no GPU (driven by
// tests/test_host.py): hashers, generators and the JSON results formatter.
//   host_check hash <xxh3|murmur3> <key> <seed>
//   host_check zipf <alpha> <lo> <hi> <seed> <n>      -> "id payload" lines
//   host_check seq <start> <n>
//   host_check json <unit> <type> <P|-> <primary> <secondary> <skew> <partition_ns> <build_ns> <probe_ns>
#include <chrono>
#include <cstdlib>
#include <iostream>
#include <memory>
#include <string>

#include "Common/Hashers.hpp"
#include "Common/Results.hpp"
#include "DataGenerator/Generators.hpp"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string cmd = argv[1];
    if (cmd == "hash" && argc == 5) {
        const int64_t key = std::stoll(argv[3]);
        const uint64_t seed = std::stoull(argv[4]);
        const std::string kind = argv[2];
        const uint64_t h = kind == "murmur3" ? phj::murmur3_fmix64(static_cast<uint64_t>(key), seed)
                                             : phj::xxh3_8(static_cast<uint64_t>(key), seed);
        std::cout << h << "\n";
        // and the reference's Hash(key, cardinality) = hash % cardinality
        Common::XXHasher x(seed);
        Common::Murmur3Hasher m(seed);
        std::cout << (kind == "murmur3" ? m.Hash(key, 1000) : x.Hash(key, 1000)) << "\n";
        return 0;
    }
    if (cmd == "zipf" && argc == 7) {
        const size_t n = std::stoull(argv[6]);
        auto t = std::make_shared<Common::Table<Common::Tuple>>(n, "zipf");
        DataGenerator::Zipf::FillTable(t, DataGenerator::Zipf::Parameters{std::stod(argv[2]),
                                                                          {std::stoll(argv[3]), std::stoll(argv[4])},
                                                                          std::stoull(argv[5]), 3});
        for (size_t i = 0; i < n; i++) std::cout << (*t)[i].id << " " << (*t)[i].payload << "\n";
        return 0;
    }
    if (cmd == "seq" && argc == 4) {
        const size_t n = std::stoull(argv[3]);
        auto t = std::make_shared<Common::Table<Common::Tuple>>(n, "seq");
        DataGenerator::Sequential::FillTable(t, DataGenerator::Sequential::Parameters{std::stoll(argv[2]), 3});
        for (size_t i = 0; i < n; i++) std::cout << (*t)[i].id << " " << (*t)[i].payload << "\n";
        return 0;
    }
    if (cmd == "json" && argc == 11) {
        Common::ResultsFormatConfiguration fc;
        fc.TimeUnit = argv[2];
        Common::Parameters p;
        p.SetParameter("PrimaryRelationSize", argv[5]);
        p.SetParameter("SecondaryRelationSize", argv[6]);
        p.SetParameter("Skew", std::to_string(std::stod(argv[7])));
        p.SetParameter("Type", argv[3]);
        if (std::string(argv[4]) != "-") p.SetParameter("NumberOfPartitions", argv[4]);
        Common::HashJoinTimingResult r(std::chrono::nanoseconds(std::stoll(argv[9])),
                                       std::chrono::nanoseconds(std::stoll(argv[10])),
                                       std::chrono::nanoseconds(std::stoll(argv[8])), p);
        Common::JSONResultsFormatter f(fc);
        f.Format(std::cout, r);
        return 0;
    }
    std::cerr << "bad command\n";
    return 2;
}
