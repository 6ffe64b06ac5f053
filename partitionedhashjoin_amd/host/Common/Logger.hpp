// Minimal severity logger to std::clog, replacing the reference's Boost.Log
// setup (src/Common/Logger.{hpp,cpp}): same severities and the same
// "LOG(logger, severity) << ..." call shape.
#pragma once

#include <iostream>
#include <sstream>
#include <string>

namespace Common {

enum SeverityLevel { trace = 0, debug, info, warning, error, critical };

std::istream& operator>>(std::istream& in, SeverityLevel& level);
std::ostream& operator<<(std::ostream& out, SeverityLevel level);
SeverityLevel GetSeverityLevelFromString(const std::string& s);

struct LoggerConfiguration {
    SeverityLevel LogLevel = debug;
};

void InitializeLogger(const LoggerConfiguration& config);
bool LogEnabled(SeverityLevel level);

struct LoggerType {
    std::string component;
};

LoggerType GetNewLogger();
void AddComponentAttributeToLogger(LoggerType& logger, const std::string& component);

class LogLine {
   public:
    LogLine(const LoggerType& logger, SeverityLevel level);
    ~LogLine();
    template <typename T>
    LogLine& operator<<(const T& v) {
        m_stream << v;
        return *this;
    }

   private:
    std::ostringstream m_stream;
};

}  // namespace Common

#define LOG(logger, sev) \
    if (!::Common::LogEnabled(sev)) {} else ::Common::LogLine((logger), (sev))
