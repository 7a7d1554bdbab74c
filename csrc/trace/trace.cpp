#include "trace.h"

#include <dlfcn.h>

#include <atomic>
#include <cstdlib>
#include <mutex>

namespace ringdp {
namespace trace {

namespace {

using push_fn = int (*)(const char*);
using pop_fn = int (*)();
using mark_fn = void (*)(const char*);
using start_fn = uint64_t (*)(const char*);
using stop_fn = void (*)(uint64_t);

struct Lib {
  push_fn push = nullptr;
  pop_fn pop = nullptr;
  mark_fn mark = nullptr;
  start_fn start = nullptr;
  stop_fn stop = nullptr;
};

std::atomic<int> g_enabled{-1};  // -1: read the environment on first use

const Lib& lib() {
  static Lib l;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                           "libroctx64.so"};
    for (const char* n : names) {
      void* h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      l.push = reinterpret_cast<push_fn>(dlsym(h, "roctxRangePushA"));
      l.pop = reinterpret_cast<pop_fn>(dlsym(h, "roctxRangePop"));
      l.mark = reinterpret_cast<mark_fn>(dlsym(h, "roctxMarkA"));
      l.start = reinterpret_cast<start_fn>(dlsym(h, "roctxRangeStartA"));
      l.stop = reinterpret_cast<stop_fn>(dlsym(h, "roctxRangeStop"));
      if (l.push && l.pop) break;
    }
  });
  return l;
}

}  // namespace

bool enabled() {
  int e = g_enabled.load(std::memory_order_relaxed);
  if (e < 0) {
    const char* v = std::getenv("RINGDP_ROCTX");
    e = (v && v[0] && v[0] != '0') ? 1 : 0;
    g_enabled.store(e, std::memory_order_relaxed);
  }
  return e == 1;
}

void set_enabled(bool on) { g_enabled.store(on ? 1 : 0, std::memory_order_relaxed); }

void push(const char* name) {
  if (enabled() && lib().push) lib().push(name);
}

void pop() {
  if (enabled() && lib().pop) lib().pop();
}

void mark(const char* msg) {
  if (enabled() && lib().mark) lib().mark(msg);
}

uint64_t start(const char* name) { return enabled() && lib().start ? lib().start(name) : 0; }

void stop(uint64_t id) {
  if (id && enabled() && lib().stop) lib().stop(id);
}

}  // namespace trace
}  // namespace ringdp
