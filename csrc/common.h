// ringdp native runtime: shared helpers (error macros, timing).
#pragma once

#include <chrono>
#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <string>

namespace ringdp {

class RingdpError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class TimeoutError : public RingdpError {
 public:
  using RingdpError::RingdpError;
};

template <typename... Args>
std::string strcat_all(Args&&... args) {
  std::ostringstream oss;
  (oss << ... << args);
  return oss.str();
}

#define RINGDP_CHECK(cond, ...)                                                        \
  do {                                                                                 \
    if (!(cond)) {                                                                     \
      throw ::ringdp::RingdpError(::ringdp::strcat_all("[ringdp] ", __FILE__, ":",     \
                                                       __LINE__, ": ", __VA_ARGS__));  \
    }                                                                                  \
  } while (0)

#define RINGDP_HIP_CHECK(expr)                                                          \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      throw ::ringdp::RingdpError(::ringdp::strcat_all("[ringdp] HIP error ",           \
                                                       hipGetErrorString(_e), " at ",   \
                                                       __FILE__, ":", __LINE__));       \
    }                                                                                   \
  } while (0)

using Clock = std::chrono::steady_clock;

inline int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             Clock::now().time_since_epoch())
      .count();
}

}  // namespace ringdp
