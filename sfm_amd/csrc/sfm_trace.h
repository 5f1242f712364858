// roctx ranges around the library's calls and LM phases, for correlating a
// rocprofv3 --marker-trace with the kernel trace (SURVEY.md §5 "Tracing /
// profiling").  Off unless SFM_ROCTX=1 (one cached getenv; no roctx call
// otherwise).  Host-side ranges: they span the enqueue (and, for calls that
// synchronise, the wait), not the GPU execution -- the kernel trace has that.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>
#include <cstdlib>

namespace sfm {
inline bool roctx_on() {
  static const bool on = [] {
    const char* e = std::getenv("SFM_ROCTX");
    return e && e[0] == '1';
  }();
  return on;
}
struct TraceRange {
  bool on;
  explicit TraceRange(const char* name) : on(roctx_on()) {
    if (on) roctxRangePushA(name);
  }
  ~TraceRange() {
    if (on) roctxRangePop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};
}  // namespace sfm

#define SFM_TRACE_CAT2(a, b) a##b
#define SFM_TRACE_CAT(a, b) SFM_TRACE_CAT2(a, b)
#define SFM_TRACE(name) ::sfm::TraceRange SFM_TRACE_CAT(sfm_trace_range_, __LINE__)(name)
