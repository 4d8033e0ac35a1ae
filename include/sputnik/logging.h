// sputnik-amd: logging / fatal-check macros with the reference's spelling.
//
// Mirrors the severity convention of reference sputnik/logging.h:8-54 and
// logging.cc:14-18: SPUTNIK_LOG(FATAL) and a failed SPUTNIK_CHECK print
// "F file:line] message" to stderr and abort(). The C++ API of this library
// aborts exactly where the reference aborts (missing metadata workspaces, no
// compatible kernel); the C-ABI in sputnik_amd.h pre-validates instead and
// returns an error code ("Errors").
#ifndef SPUTNIK_LOGGING_H_
#define SPUTNIK_LOGGING_H_

#include <cstdio>
#include <cstdlib>
#include <sstream>

namespace sputnik {

constexpr int INFO = 0;
constexpr int WARNING = 1;
constexpr int ERROR = 2;
constexpr int FATAL = 3;

namespace internal {

// Collects one message; emits it (and aborts on FATAL) when destroyed.
class LogMessage : public std::ostringstream {
 public:
  LogMessage(const char *file, int line, int severity)
      : file_(file), line_(line), severity_(severity) {}
  ~LogMessage() {
    std::fprintf(stderr, "%c %s:%d] %s\n", "IWEF"[severity_ & 3], file_,
                 line_, str().c_str());
    if (severity_ == FATAL) std::abort();
  }

 private:
  const char *file_;
  int line_;
  int severity_;
};

}  // namespace internal
}  // namespace sputnik

#define SPUTNIK_LOG(severity) \
  ::sputnik::internal::LogMessage(__FILE__, __LINE__, ::sputnik::severity)

#define SPUTNIK_CHECK(condition) \
  if (!(condition)) SPUTNIK_LOG(FATAL) << "Check failed: " #condition " "

#define SPUTNIK_CHECK_EQ(a, b) SPUTNIK_CHECK((a) == (b))
#define SPUTNIK_CHECK_NE(a, b) SPUTNIK_CHECK((a) != (b))
#define SPUTNIK_CHECK_LE(a, b) SPUTNIK_CHECK((a) <= (b))
#define SPUTNIK_CHECK_LT(a, b) SPUTNIK_CHECK((a) < (b))
#define SPUTNIK_CHECK_GE(a, b) SPUTNIK_CHECK((a) >= (b))
#define SPUTNIK_CHECK_GT(a, b) SPUTNIK_CHECK((a) > (b))

#endif  // SPUTNIK_LOGGING_H_
