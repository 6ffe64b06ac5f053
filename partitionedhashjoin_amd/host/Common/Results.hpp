// Phase timing and result rendering of the reference (src/Common/Results.hpp):
// Parameters, HashJoinTimingResult, IHashJoinTimer / NoOpHashJoinTimer /
// HashJoinTimer (same phase semantics, including the NoPartitioning quirk that
// SetProbePhaseEnd measures from the build start, Results.hpp:202), and a JSON
// formatter whose output has the layout Boost.PropertyTree's write_json gives
// the reference (results/*/partitions_*.txt): 4-space indent, string values,
// keys `id`, `parameters.*`, `results.{partition,build,probe}`. New values go
// into an appended top-level `device` object (matches, device_total_us, ...),
// never into `results`, whose values scripts/generate.sh pastes as rows.
#pragma once

#include <chrono>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <ostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "Common/Configuration.hpp"

namespace Common {

class Parameters {
   public:
    using StorageType = std::map<std::string, std::string>;
    void SetParameter(std::string key, std::string value) { m_values[key] = value; }
    StorageType::const_iterator begin() const { return m_values.begin(); }
    StorageType::const_iterator end() const { return m_values.end(); }

   private:
    StorageType m_values;
};

class HashJoinTimingResult {
   public:
    HashJoinTimingResult() = default;
    HashJoinTimingResult(std::chrono::nanoseconds build, std::chrono::nanoseconds probe,
                         std::chrono::nanoseconds partitioning, const Parameters& parameters)
        : m_parameters(parameters), m_buildPhase(build), m_probePhase(probe), m_partitioningPhase(partitioning) {}

    void SetBuildPhaseDuration(std::chrono::nanoseconds d) { m_buildPhase = d; }
    void SetProbePhaseDuration(std::chrono::nanoseconds d) { m_probePhase = d; }
    void SetPartitioningPhaseDuration(std::chrono::nanoseconds d) { m_partitioningPhase = d; }
    void SetParameters(const Parameters& p) { m_parameters = p; }
    // additive result fields (rendered after partition/build/probe, in insertion order)
    void AddResult(const std::string& key, const std::string& value) { m_extra.emplace_back(key, value); }

    std::chrono::nanoseconds GetBuildPhaseDuration() const { return m_buildPhase; }
    std::chrono::nanoseconds GetProbePhaseDuration() const { return m_probePhase; }
    std::chrono::nanoseconds GetPartitioningPhaseDuration() const { return m_partitioningPhase; }
    const Parameters& GetParameters() const { return m_parameters; }
    const std::vector<std::pair<std::string, std::string>>& GetExtraResults() const { return m_extra; }

   private:
    Parameters m_parameters;
    std::chrono::nanoseconds m_buildPhase{0};
    std::chrono::nanoseconds m_probePhase{0};
    std::chrono::nanoseconds m_partitioningPhase{0};
    std::vector<std::pair<std::string, std::string>> m_extra;
};

class IHashJoinTimer {
   public:
    // continuous segments (not thread-safe)
    virtual void SetBuildPhaseBegin() = 0;
    virtual void SetBuildPhaseEnd() = 0;
    virtual void SetPartitioningPhaseBegin() = 0;
    virtual void SetPartitioningPhaseEnd() = 0;
    virtual void SetProbePhaseBegin() = 0;
    virtual void SetProbePhaseEnd() = 0;
    // discontinuous segments (here: device-measured phase times)
    virtual void SetBuildPhaseDuration(std::chrono::nanoseconds duration) = 0;
    virtual void SetProbePhaseDuration(std::chrono::nanoseconds duration) = 0;
    virtual void SetPartitionPhaseDuration(std::chrono::nanoseconds duration) = 0;
    // additive: extra result fields for the JSON output
    virtual void AddResult(const std::string&, const std::string&) {}
    virtual HashJoinTimingResult GetResult() = 0;
    virtual ~IHashJoinTimer() = default;
};

class NoOpHashJoinTimer final : public IHashJoinTimer {
   public:
    void SetBuildPhaseBegin() override {}
    void SetBuildPhaseEnd() override {}
    void SetPartitioningPhaseBegin() override {}
    void SetPartitioningPhaseEnd() override {}
    void SetProbePhaseBegin() override {}
    void SetProbePhaseEnd() override {}
    void SetBuildPhaseDuration(std::chrono::nanoseconds) override {}
    void SetProbePhaseDuration(std::chrono::nanoseconds) override {}
    void SetPartitionPhaseDuration(std::chrono::nanoseconds) override {}
    HashJoinTimingResult GetResult() override { return HashJoinTimingResult(); }
};

class HashJoinTimer final : public IHashJoinTimer {
   public:
    explicit HashJoinTimer(const Parameters& parameters) : m_parameters(parameters) {}

    void SetBuildPhaseBegin() override { m_buildStart = clock::now(); }
    void SetBuildPhaseEnd() override { m_buildTime = clock::now() - m_buildStart; }
    void SetPartitioningPhaseBegin() override { m_partitioningStart = clock::now(); }
    void SetPartitioningPhaseEnd() override { m_partitioningTime = clock::now() - m_partitioningStart; }
    void SetProbePhaseBegin() override { m_probeStart = clock::now(); }
    // measured from the build start, as the reference does (Results.hpp:202)
    void SetProbePhaseEnd() override { m_probeTime = clock::now() - m_buildStart; }
    void SetBuildPhaseDuration(std::chrono::nanoseconds d) override { m_buildTime = d; }
    void SetProbePhaseDuration(std::chrono::nanoseconds d) override { m_probeTime = d; }
    void SetPartitionPhaseDuration(std::chrono::nanoseconds d) override { m_partitioningTime = d; }
    void AddResult(const std::string& k, const std::string& v) override { m_extra.emplace_back(k, v); }

    HashJoinTimingResult GetResult() override {
        HashJoinTimingResult r(m_buildTime, m_probeTime, m_partitioningTime, m_parameters);
        for (const auto& kv : m_extra) r.AddResult(kv.first, kv.second);
        return r;
    }

   private:
    using clock = std::chrono::steady_clock;
    Parameters m_parameters;
    std::chrono::nanoseconds m_buildTime{0}, m_probeTime{0}, m_partitioningTime{0};
    clock::time_point m_buildStart, m_probeStart, m_partitioningStart;
    std::vector<std::pair<std::string, std::string>> m_extra;
};

class IResultsFormatter {
   public:
    virtual void Format(std::basic_ostream<char>& stream, const HashJoinTimingResult& result) = 0;
    virtual ~IResultsFormatter() = default;
};

class IResultsRenderer {
   public:
    virtual void Render(std::shared_ptr<IResultsFormatter> formatter, const HashJoinTimingResult& result) = 0;
    virtual ~IResultsRenderer() = default;
};

class JSONResultsFormatter final : public IResultsFormatter {
   public:
    explicit JSONResultsFormatter(const ResultsFormatConfiguration& config) : m_config(config) {}

    void Format(std::basic_ostream<char>& stream, const HashJoinTimingResult& r) override {
        std::vector<std::pair<std::string, std::string>> params(r.GetParameters().begin(), r.GetParameters().end());
        const std::vector<std::pair<std::string, std::string>> results = {
            {"partition", Cast(r.GetPartitioningPhaseDuration())},
            {"build", Cast(r.GetBuildPhaseDuration())},
            {"probe", Cast(r.GetProbePhaseDuration())}};
        const auto& extra = r.GetExtraResults();
        stream << "{\n    \"id\": \"hashjointimingresult\",\n";
        WriteObject(stream, "parameters", params, true);
        // `results` holds exactly the reference's three phases: scripts/generate.sh
        // pastes every `.results` value into figure.dat (generate.sh:25)
        WriteObject(stream, "results", results, !extra.empty());
        if (!extra.empty()) WriteObject(stream, "device", extra, false);
        stream << "}\n";
    }

    std::string Cast(std::chrono::nanoseconds d) const {
        std::ostringstream s;
        if (m_config.TimeUnit == "ns") s << d.count();
        else if (m_config.TimeUnit == "us") s << std::chrono::duration_cast<std::chrono::microseconds>(d).count();
        else if (m_config.TimeUnit == "ms") s << std::chrono::duration_cast<std::chrono::milliseconds>(d).count();
        else if (m_config.TimeUnit == "s") s << std::chrono::duration_cast<std::chrono::seconds>(d).count();
        else
            throw std::runtime_error("JSONResultsFormatter::CastDurationToString: unrecognized duration unit: " +
                                     m_config.TimeUnit);
        return s.str();
    }

   private:
    static std::string Escape(const std::string& v) {
        std::string o;
        for (char ch : v) {
            if (ch == '"' || ch == '\\') o.push_back('\\');
            o.push_back(ch);
        }
        return o;
    }
    static void WriteObject(std::basic_ostream<char>& s, const char* name,
                            const std::vector<std::pair<std::string, std::string>>& kv, bool comma) {
        s << "    \"" << name << "\": {\n";
        for (size_t i = 0; i < kv.size(); i++) {
            s << "        \"" << Escape(kv[i].first) << "\": \"" << Escape(kv[i].second) << "\"";
            s << (i + 1 < kv.size() ? ",\n" : "\n");
        }
        s << "    }" << (comma ? ",\n" : "\n");
    }
    const ResultsFormatConfiguration m_config;
};

class FileResultsRenderer final : public IResultsRenderer {
   public:
    explicit FileResultsRenderer(const OutputConfiguration& config) : m_file(config.File.Name) {
        if (!m_file) throw std::runtime_error("FileResultsRenderer: cannot open " + config.File.Name);
    }
    void Render(std::shared_ptr<IResultsFormatter> formatter, const HashJoinTimingResult& result) override {
        formatter->Format(m_file, result);
        m_file.flush();
    }

   private:
    std::ofstream m_file;
};

inline std::shared_ptr<IResultsFormatter> SelectResultsFormatter(const Configuration& config) {
    if (config.OutputFormatConfig.Format == ResultsFormat::JSON)
        return std::make_shared<JSONResultsFormatter>(config.OutputFormatConfig);
    throw std::runtime_error("Unrecognized results format.");
}

inline std::shared_ptr<IResultsRenderer> SelectResultsRenderer(const Configuration& config) {
    if (config.OutputConfig.Type == OutputType::File) return std::make_shared<FileResultsRenderer>(config.OutputConfig);
    throw std::runtime_error("Unrecognized output type.");
}

}  // namespace Common
