// phjoin — the reference's benchmark CLI (src/main.cpp, src/Arguments.hpp)
// running the join on an MI355X through the C ABI.
//
// Same flags, defaults, validation and output as the reference:
//   --primary 10000000 --secondary 200000000 --skew 1.05 --log debug
//   --join no-partitioning|radix-partitioning (required) --format json
//   -u/--unit ns|us|ms|s (ms) -o/--output file -f/--filename hashjoin.txt
//   -p/--partitions P (radix only; default 32)
// Additive flags:
//   --device N            HIP device (default 0)
//   --hash xxh3|murmur3   (default xxh3, as XXHasher)
//   --radix-bits B0[,B1]  power-of-two radix partitioning (e.g. 8,8) instead of hash % P
//   --seed S              data generator seed (default 20240601)
//   --hash-seed S         hasher seed (default: random, as the reference)
//   --generate host|device  where the relations are generated (default host)
//   --table-ratio X       no-partitioning: table slots per build tuple
//   --gpus N | --devices a,b,..  several devices (multi-GPU join over RCCL)
//   --exchange rccl|local  force the multi-GPU path (RCCL world of one / device copies)
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "Common/Configuration.hpp"
#include "Common/Hashers.hpp"
#include "Common/Logger.hpp"
#include "Common/Results.hpp"
#include "Common/Table.hpp"
#include "DataGenerator/Generators.hpp"
#include "Gpu/HashJoin.hpp"

namespace {

const char* kHelp =
    "Allowed options:\n"
    "  -h [ --help ]                       Help screen\n"
    "  --primary arg (=10000000)           Size of the primary relation.\n"
    "  --secondary arg (=200000000)        Size of the secondary relation.\n"
    "  --skew arg (=1.05)                  Parameter of skew for Zipf distribution used for the\n"
    "                                      generation of tuples for secondary relation.\n"
    "  --log arg (=debug)                  Logging level. One of {trace, debug, info, error, critical}.\n"
    "  --join arg                          Type of join algorithm: either no-partitioning or\n"
    "                                      radix-partitioning.\n"
    "  --format arg (=json)                Format of the output. Currently only JSON is supported.\n"
    "  -u [ --unit ] arg (=ms)             Duration unit of the timing output. One of {ns, us, ms, s}.\n"
    "  -o [ --output ] arg (=file)         Type of the output. Currently only file is supported.\n"
    "  -f [ --filename ] arg (=hashjoin.txt)\n"
    "                                      Name of the file if output type is file.\n"
    "  -p [ --partitions ] arg             Number of partitions for algorithms using partitioning.\n"
    "MI355X options:\n"
    "  --device arg (=0)                   HIP device.\n"
    "  --hash arg (=xxh3)                  xxh3 | murmur3.\n"
    "  --radix-bits arg                    B0[,B1]: power-of-two radix partitioning, one or two passes.\n"
    "  --seed arg (=20240601)              Seed of the relation generators.\n"
    "  --hash-seed arg                     Hasher seed (default: random).\n"
    "  --generate arg (=host)              host | device.\n"
    "  --table-ratio arg                   No-partitioning table slots per build tuple.\n"
    "  --materialize arg (=off)            on | off: return the joined rows (Table<JoinedTuple>).\n"
    "  --gpus arg (=1)                     Devices --device .. --device+N-1: range-sharded relations,\n"
    "                                      RCCL exchange of the partitioned build side.\n"
    "  --devices arg                       Explicit device list a,b,... (instead of --gpus).\n"
    "  --exchange arg                      rccl | local: force the multi-GPU path (rccl on one device is\n"
    "                                      an RCCL world of one; local = device copies, devices may repeat).\n";

// --materialize on: the rows Run() returned (count, and a checksum of their
// columns so a caller can compare runs without the rows themselves)
void report_rows(const Common::Table<Common::JoinedTuple>& rows, Common::IHashJoinTimer& timer, bool materialize) {
    if (!materialize) return;
    uint64_t sum = 0;
    for (size_t i = 0; i < rows.GetSize(); i++)
        sum += static_cast<uint64_t>(rows[i].id) * 3 + static_cast<uint64_t>(rows[i].payloadA) * 5 +
               static_cast<uint64_t>(rows[i].payloadB) * 7;
    timer.AddResult("rows", std::to_string(rows.GetSize()));
    timer.AddResult("rows_checksum", std::to_string(sum));
}

template <typename T>
T parse_number(const std::string& name, const std::string& v) {
    std::istringstream s(v);
    T out{};
    s >> out;
    if (!s || !s.eof()) throw std::invalid_argument("the argument ('" + v + "') for option '--" + name + "' is invalid");
    return out;
}

// Boost.program_options-like parsing: --name value, --name=value, -x value.
Common::Configuration parseArguments(int argc, char** argv) {
    static const std::map<std::string, std::string> shortNames = {
        {"-u", "unit"}, {"-o", "output"}, {"-f", "filename"}, {"-p", "partitions"}, {"-h", "help"}};
    static const std::set<std::string> known = {"help", "primary", "secondary", "skew", "log", "join", "format",
                                                "unit", "output", "filename", "partitions", "device", "gpus", "devices", "exchange", "hash",
                                                "radix-bits", "seed", "hash-seed", "generate", "table-ratio",
                                                "materialize"};
    Common::Configuration c{};
    c.OutputFormatConfig.TimeUnit = "ms";
    c.OutputConfig.File.Name = "hashjoin.txt";
    std::map<std::string, std::string> vm;
    try {
        for (int i = 1; i < argc; i++) {
            std::string a = argv[i], name, value;
            bool has_value = false;
            if (a.rfind("--", 0) == 0) {
                name = a.substr(2);
                const auto eq = name.find('=');
                if (eq != std::string::npos) {
                    value = name.substr(eq + 1);
                    name = name.substr(0, eq);
                    has_value = true;
                }
            } else if (shortNames.count(a)) {
                name = shortNames.at(a);
            } else {
                throw std::invalid_argument("unrecognised option '" + a + "'");
            }
            if (!known.count(name)) throw std::invalid_argument("unrecognised option '--" + name + "'");
            if (name == "help") {
                std::cout << kHelp << "\n";
                std::exit(0);
            }
            if (!has_value) {
                if (i + 1 >= argc) throw std::invalid_argument("the required argument for option '--" + name + "' is missing");
                value = argv[++i];
            }
            if (vm.count(name)) throw std::invalid_argument("option '--" + name + "' cannot be specified more than once");
            vm[name] = value;
        }
        if (!vm.count("join")) throw std::invalid_argument("the option '--join' is required but missing");
        c.JoinType = Common::GetJoinAlgorithmTypeFromString(vm["join"]);
        if (vm.count("primary")) c.PrimaryRelationSize = parse_number<size_t>("primary", vm["primary"]);
        if (vm.count("secondary")) c.SecondaryRelationSize = parse_number<size_t>("secondary", vm["secondary"]);
        if (vm.count("skew")) c.SkewParameter = parse_number<double>("skew", vm["skew"]);
        if (vm.count("log")) c.LoggerConfig.LogLevel = Common::GetSeverityLevelFromString(vm["log"]);
        if (vm.count("format")) c.OutputFormatConfig.Format = Common::GetResultsFormatFromString(vm["format"]);
        if (vm.count("unit")) c.OutputFormatConfig.TimeUnit = vm["unit"];
        if (vm.count("output")) c.OutputConfig.Type = Common::GetOutputTypeFromString(vm["output"]);
        if (vm.count("filename")) c.OutputConfig.File.Name = vm["filename"];
        if (vm.count("partitions"))
            c.RadixClusteringConfig.NumberOfPartitions = parse_number<size_t>("partitions", vm["partitions"]);
        if (vm.count("device")) c.GpuConfig.Device = parse_number<int>("device", vm["device"]);
        if (vm.count("materialize")) {
            if (vm["materialize"] == "on") c.GpuConfig.Materialize = true;
            else if (vm["materialize"] != "off")
                throw std::invalid_argument("the argument ('" + vm["materialize"] + "') for option '--materialize' is invalid");
        }
        c.GpuConfig.Hash = PHJ_HASH_XXH3;
        if (vm.count("hash")) {
            if (vm["hash"] == "xxh3" || vm["hash"] == "xxhash") c.GpuConfig.Hash = PHJ_HASH_XXH3;
            else if (vm["hash"] == "murmur3") c.GpuConfig.Hash = PHJ_HASH_MURMUR3;
            else throw std::invalid_argument("the argument ('" + vm["hash"] + "') for option '--hash' is invalid");
            c.GpuConfig.HashSet = true;
        }
        if (vm.count("radix-bits")) {
            const std::string v = vm["radix-bits"];
            const auto comma = v.find(',');
            c.GpuConfig.RadixBits[0] = parse_number<unsigned>("radix-bits", v.substr(0, comma));
            c.GpuConfig.RadixBits[1] = comma == std::string::npos ? 0 : parse_number<unsigned>("radix-bits", v.substr(comma + 1));
            if (c.GpuConfig.RadixBits[0] < 1 || c.GpuConfig.RadixBits[0] > 11 || c.GpuConfig.RadixBits[1] > 11)
                throw std::invalid_argument("--radix-bits: each pass takes 1..11 bits (second may be 0)");
        }
        if (vm.count("seed")) c.GpuConfig.Seed = parse_number<uint64_t>("seed", vm["seed"]);
        if (vm.count("hash-seed")) {
            c.GpuConfig.HashSeed = parse_number<uint64_t>("hash-seed", vm["hash-seed"]);
            c.GpuConfig.HashSeedSet = true;
        }
        if (vm.count("generate")) {
            if (vm["generate"] == "device") c.GpuConfig.GenerateOnDevice = true;
            else if (vm["generate"] != "host")
                throw std::invalid_argument("the argument ('" + vm["generate"] + "') for option '--generate' is invalid");
        }
        if (vm.count("table-ratio")) c.GpuConfig.TableRatio = parse_number<double>("table-ratio", vm["table-ratio"]);
        if (vm.count("gpus") && vm.count("devices"))
            throw std::invalid_argument("--gpus and --devices are mutually exclusive");
        if (vm.count("gpus")) {
            const int n = parse_number<int>("gpus", vm["gpus"]);
            if (n < 1 || n > 16) throw std::invalid_argument("--gpus takes 1..16");
            for (int i = 0; i < n; i++) c.GpuConfig.Devices.push_back(c.GpuConfig.Device + i);
        }
        if (vm.count("devices")) {
            std::string v = vm["devices"];
            size_t pos = 0;
            while (pos <= v.size()) {
                const size_t comma = v.find(',', pos);
                const std::string item = v.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos);
                c.GpuConfig.Devices.push_back(parse_number<int>("devices", item));
                if (comma == std::string::npos) break;
                pos = comma + 1;
            }
            if (c.GpuConfig.Devices.empty() || c.GpuConfig.Devices.size() > 16)
                throw std::invalid_argument("--devices takes 1..16 device ids");
        }
        if (vm.count("exchange")) {
            if (vm["exchange"] == "rccl") c.GpuConfig.ContextFlags = PHJ_CTX_EXCHANGE;
            else if (vm["exchange"] == "local") c.GpuConfig.ContextFlags = PHJ_CTX_LOCAL;
            else throw std::invalid_argument("the argument ('" + vm["exchange"] + "') for option '--exchange' is invalid");
        }
        if (c.GpuConfig.Materialize && (c.GpuConfig.Devices.size() > 1 || c.GpuConfig.ContextFlags))
            throw std::invalid_argument("--materialize on runs on one device");
        // validateParsedConfiguration (src/Arguments.hpp:7-18)
        c.OutputConfig.Validate();
        c.OutputFormatConfig.Validate();
        if (c.JoinType != Common::JoinAlgorithmType::RadixParitioning && (vm.count("partitions") || vm.count("radix-bits")))
            throw std::invalid_argument(
                "validateParsedConfiguration: number of partitions can be specified only for RadixParitioning.");
        if (vm.count("partitions") && vm.count("radix-bits"))
            throw std::invalid_argument("--partitions and --radix-bits are mutually exclusive");
    } catch (std::exception& e) {
        std::cout << e.what() << "\n\n" << kHelp << "\n";
        std::exit(1);
    }
    return c;
}

Common::Parameters baseParameters(const Common::Configuration& c, const char* type) {
    Common::Parameters p;
    p.SetParameter("PrimaryRelationSize", std::to_string(c.PrimaryRelationSize));
    p.SetParameter("SecondaryRelationSize", std::to_string(c.SecondaryRelationSize));
    p.SetParameter("Skew", std::to_string(c.SkewParameter));
    p.SetParameter("Type", type);
    return p;
}

}  // namespace

int main(int argc, char** argv) {
    Common::Configuration configuration = parseArguments(argc, argv);
    Common::InitializeLogger(configuration.LoggerConfig);
    auto logger = Common::GetNewLogger();
    Common::AddComponentAttributeToLogger(logger, "main");

    std::shared_ptr<Common::IResultsFormatter> resultsFormatter = Common::SelectResultsFormatter(configuration);
    std::shared_ptr<Common::IResultsRenderer> resultsRenderer;
    try {
        resultsRenderer = Common::SelectResultsRenderer(configuration);
    } catch (std::exception& e) {
        LOG(logger, Common::error) << e.what();
        return 1;
    }

    LOG(logger, Common::info) << "Starting running tests.";
    std::shared_ptr<Gpu::Device> device;
    try {
        const auto& g = configuration.GpuConfig;
        if (g.Devices.size() > 1 || g.ContextFlags)
            device = std::make_shared<Gpu::Device>(g.Devices.empty() ? std::vector<int>{g.Device} : g.Devices,
                                                   g.ContextFlags);
        else
            device = std::make_shared<Gpu::Device>(g.Devices.empty() ? g.Device : g.Devices[0]);
    } catch (std::exception& e) {
        LOG(logger, Common::error) << "No usable HIP device: " << e.what();
        return 1;
    }

    // generateTables (src/main.cpp:35-79): R Sequential from 1, S Zipf over [1, |R|]
    const size_t nR = configuration.PrimaryRelationSize, nS = configuration.SecondaryRelationSize;
    LOG(logger, Common::debug) << "Generating primary relation with size " << nR << " and secondary relation with size "
                               << nS << ".";
    std::shared_ptr<Common::Table<Common::Tuple>> tableA, tableB;
    if (configuration.GpuConfig.GenerateOnDevice) {
        device->Check(phj_relation_generate_sequential(device->Get(), PHJ_SIDE_BUILD, nR, 1, 0));
        device->Check(phj_relation_generate_zipf(device->Get(), PHJ_SIDE_PROBE, nS, configuration.SkewParameter, 1,
                                                 static_cast<int64_t>(nR), configuration.GpuConfig.Seed, 0));
    } else {
        tableA = std::make_shared<Common::Table<Common::Tuple>>(nR, Common::generate_uuid());
        tableB = std::make_shared<Common::Table<Common::Tuple>>(nS, Common::generate_uuid());
        DataGenerator::Sequential::FillTable(tableA, DataGenerator::Sequential::Parameters{1});
        DataGenerator::Zipf::FillTable(
            tableB, DataGenerator::Zipf::Parameters{configuration.SkewParameter, {1, static_cast<int64_t>(nR)},
                                                    configuration.GpuConfig.Seed});
    }
    LOG(logger, Common::debug) << "Generation of relations finished.";

    const uint64_t hashSeed =
        configuration.GpuConfig.HashSeedSet ? configuration.GpuConfig.HashSeed : Common::internal::random_seed();
    Common::HashJoinTimingResult joinResults;
    try {
        switch (configuration.JoinType) {
            case Common::JoinAlgorithmType::NoPartitioning: {
                LOG(logger, Common::debug) << "Executing NoPartitionHashJoin algorithm.";
                auto params = baseParameters(configuration, "NoPartitioning");
                auto timer = std::make_shared<Common::HashJoinTimer>(params);
                auto run = [&](auto hasher) {
                    using H = decltype(hasher);
                    HashTables::LinearProbingFactory<Common::Tuple, 3, H> factory(HashTables::LinearProbingConfiguration{},
                                                                                  hasher);
                    Gpu::NoPartitioning::HashJoiner<decltype(factory)> joiner(configuration.NoPartitioningConfig, device,
                                                                             factory, configuration.GpuConfig);
                    auto joined = tableA ? joiner.Run(tableA, tableB, timer) : joiner.RunResident(timer);
                    report_rows(*joined, *timer, configuration.GpuConfig.Materialize);
                };
                if (configuration.GpuConfig.Hash == PHJ_HASH_MURMUR3) run(Common::Murmur3Hasher(hashSeed));
                else run(Common::XXHasher(hashSeed));
                joinResults = timer->GetResult();
                LOG(logger, Common::debug) << "Finished executing NoPartitionHashJoin algorithm.";
                break;
            }
            case Common::JoinAlgorithmType::RadixParitioning: {
                LOG(logger, Common::debug) << "Executing Radix Clustering join algorithm.";
                auto params = baseParameters(configuration, "RadixParitioning");
                if (configuration.GpuConfig.RadixBits[0] > 0) {
                    const unsigned bits = configuration.GpuConfig.RadixBits[0] + configuration.GpuConfig.RadixBits[1];
                    params.SetParameter("NumberOfPartitions", std::to_string(1ull << bits));
                    params.SetParameter("RadixBits", std::to_string(configuration.GpuConfig.RadixBits[0]) + "," +
                                                         std::to_string(configuration.GpuConfig.RadixBits[1]));
                } else {
                    params.SetParameter("NumberOfPartitions",
                                        std::to_string(configuration.RadixClusteringConfig.NumberOfPartitions));
                }
                auto timer = std::make_shared<Common::HashJoinTimer>(params);
                auto run = [&](auto hasher) {
                    using H = decltype(hasher);
                    HashTables::LinearProbingFactory<Common::Tuple, 3, H> factory(HashTables::LinearProbingConfiguration{},
                                                                                  hasher);
                    Gpu::RadixClustering::HashJoiner<decltype(factory), H> joiner(
                        configuration.RadixClusteringConfig, device, hasher, factory, configuration.GpuConfig);
                    auto joined = tableA ? joiner.Run(tableA, tableB, timer) : joiner.RunResident(timer);
                    report_rows(*joined, *timer, configuration.GpuConfig.Materialize);
                };
                if (configuration.GpuConfig.Hash == PHJ_HASH_MURMUR3) run(Common::Murmur3Hasher(hashSeed));
                else run(Common::XXHasher(hashSeed));
                joinResults = timer->GetResult();
                LOG(logger, Common::debug) << "Finished executing Radix Clustering join algorithm.";
                break;
            }
        }
    } catch (std::exception& e) {
        LOG(logger, Common::error) << "Hash join algorithm stopped due to exception begin raised: " << e.what();
        return 1;
    }

    resultsRenderer->Render(resultsFormatter, joinResults);
    LOG(logger, Common::info) << "Finished running tests.";
    return 0;
}
