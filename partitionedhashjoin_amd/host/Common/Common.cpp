// Logger, uuid and enum parsing for the host driver.
#include <atomic>
#include <chrono>
#include <ctime>
#include <iomanip>
#include <mutex>
#include <random>
#include <stdexcept>

#include "Common/Configuration.hpp"
#include "Common/Logger.hpp"
#include "Common/Table.hpp"

namespace Common {

namespace {
std::atomic<int> g_level{debug};
std::mutex g_log_mutex;

const char* severity_name(SeverityLevel l) {
    switch (l) {
        case trace: return "trace";
        case debug: return "debug";
        case info: return "info";
        case warning: return "warning";
        case error: return "error";
        case critical: return "critical";
    }
    return "unknown";
}
}  // namespace

SeverityLevel GetSeverityLevelFromString(const std::string& s) {
    if (s == "trace") return trace;
    if (s == "debug") return debug;
    if (s == "info") return info;
    if (s == "warning") return warning;
    if (s == "error") return error;
    if (s == "critical") return critical;
    throw std::invalid_argument("Unrecognized log level: " + s + ".");
}

std::istream& operator>>(std::istream& in, SeverityLevel& level) {
    std::string s;
    in >> s;
    level = GetSeverityLevelFromString(s);
    return in;
}

std::ostream& operator<<(std::ostream& out, SeverityLevel level) { return out << severity_name(level); }

void InitializeLogger(const LoggerConfiguration& config) { g_level = config.LogLevel; }

bool LogEnabled(SeverityLevel level) { return static_cast<int>(level) >= g_level.load(); }

LoggerType GetNewLogger() { return LoggerType{}; }

void AddComponentAttributeToLogger(LoggerType& logger, const std::string& component) {
    logger.component = component;
}

LogLine::LogLine(const LoggerType& logger, SeverityLevel level) {
    const auto now = std::chrono::system_clock::now();
    const std::time_t t = std::chrono::system_clock::to_time_t(now);
    std::tm tm{};
    localtime_r(&t, &tm);
    m_stream << "[" << std::put_time(&tm, "%Y-%m-%d %H:%M:%S") << "] [" << severity_name(level) << "]";
    if (!logger.component.empty()) m_stream << " [" << logger.component << "]";
    m_stream << " ";
}

LogLine::~LogLine() {
    std::lock_guard<std::mutex> lock(g_log_mutex);
    std::clog << m_stream.str() << std::endl;
}

std::string generate_uuid() {
    static std::mutex mu;
    static std::mt19937_64 gen{std::random_device{}()};
    std::lock_guard<std::mutex> lock(mu);
    const uint64_t a = gen(), b = gen();
    std::ostringstream s;
    s << std::hex << std::setfill('0') << std::setw(8) << (a >> 32) << "-" << std::setw(4) << ((a >> 16) & 0xffff)
      << "-4" << std::setw(3) << (a & 0xfff) << "-" << std::setw(4) << ((b >> 48 & 0x3fff) | 0x8000) << "-"
      << std::setw(12) << (b & 0xffffffffffffULL);
    return s.str();
}

// ---- Configuration enums (src/Common/Configuration.cpp:4-84) ----
JoinAlgorithmType GetJoinAlgorithmTypeFromString(const std::string& algorithmType) {
    if (algorithmType == "no-partitioning") return JoinAlgorithmType::NoPartitioning;
    if (algorithmType == "radix-partitioning") return JoinAlgorithmType::RadixParitioning;
    throw std::runtime_error("Unrecognized join algorithm type: " + algorithmType + ".");
}

std::istream& operator>>(std::istream& in, JoinAlgorithmType& obj) {
    std::string s;
    in >> s;
    obj = GetJoinAlgorithmTypeFromString(s);
    return in;
}

std::ostream& operator<<(std::ostream& os, JoinAlgorithmType t) {
    switch (t) {
        case JoinAlgorithmType::NoPartitioning: return os << "no-partitioning";
        case JoinAlgorithmType::RadixParitioning: return os << "radix-partitioning";
    }
    return os << static_cast<int>(t);
}

ResultsFormat GetResultsFormatFromString(const std::string& s) {
    if (s == "json") return ResultsFormat::JSON;
    throw std::runtime_error("Unrecognized results format: " + s + ".");
}

std::istream& operator>>(std::istream& in, ResultsFormat& obj) {
    std::string s;
    in >> s;
    obj = GetResultsFormatFromString(s);
    return in;
}

std::ostream& operator<<(std::ostream& os, ResultsFormat f) {
    if (f == ResultsFormat::JSON) return os << "json";
    return os << static_cast<int>(f);
}

OutputType GetOutputTypeFromString(const std::string& s) {
    if (s == "file") return OutputType::File;
    throw std::runtime_error("Unrecognized output type: " + s + ".");
}

std::istream& operator>>(std::istream& in, OutputType& obj) {
    std::string s;
    in >> s;
    obj = GetOutputTypeFromString(s);
    return in;
}

std::ostream& operator<<(std::ostream& os, OutputType t) {
    if (t == OutputType::File) return os << "file";
    return os << static_cast<int>(t);
}

void OutputConfiguration::Validate() const {
    if (Type == OutputType::File && File.Name.empty())
        throw std::invalid_argument("OutputConfiguration::Validate: empty configuration filename specified.");
}

void ResultsFormatConfiguration::Validate() const {
    for (const char* u : {"ns", "us", "ms", "s"})
        if (TimeUnit == u) return;
    throw std::invalid_argument("ResultsFormatConfiguration::Validate: Unrecognized time unit: " + TimeUnit);
}

}  // namespace Common
