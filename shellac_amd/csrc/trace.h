// Timeline markers for rocprofv3 ("roctracer markers around HIP
// batches"). ROCTX ranges from rocprofiler-sdk-roctx, recorded by
// `rocprofv3 --marker-trace --kernel-trace ...`. Off unless SHELLAC_TRACE=1 (or
// trace_enable(true)), so the serving path pays one predictable branch.
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

#include <atomic>
#include <cstdlib>

namespace shellac {

inline std::atomic<bool>& trace_flag() {
  static std::atomic<bool> on{[] {
    const char* e = std::getenv("SHELLAC_TRACE");
    return e && *e && *e != '0';
  }()};
  return on;
}
inline bool trace_on() { return trace_flag().load(std::memory_order_relaxed); }
inline void trace_enable(bool on) { trace_flag().store(on); }
inline void trace_push(const char* name) {
  if (trace_on()) roctxRangePushA(name);
}
inline void trace_pop() {
  if (trace_on()) roctxRangePop();
}
inline void trace_mark(const char* name) {
  if (trace_on()) roctxMarkA(name);
}

// RAII range; the flag is sampled once so push/pop always pair.
class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(trace_on()) {
    if (on_) roctxRangePushA(name);
  }
  ~TraceRange() {
    if (on_) roctxRangePop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

}  // namespace shellac
