// roctx ranges/markers for rocprofv3 --marker-trace (SURVEY.md §5 "Tracing / profiling").
// The roctx library is dlopen'ed on first use so the extension has no hard dependency on the
// profiler SDK; with tracing disabled (default; RINGDP_ROCTX=1 or set_enabled(true) turns it on)
// every call is one relaxed atomic load.
#pragma once

#include <cstdint>
#include <string>

namespace ringdp {
namespace trace {

bool enabled();
void set_enabled(bool on);
void push(const char* name);
void pop();
void mark(const char* msg);
uint64_t start(const char* name);
void stop(uint64_t id);

struct Range {
  explicit Range(const char* name) : on_(enabled()) {
    if (on_) push(name);
  }
  ~Range() {
    if (on_) pop();
  }
  bool on_;
};

}  // namespace trace
}  // namespace ringdp
