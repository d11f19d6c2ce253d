// roctx ranges for the per-frame stages: visible in
// `rocprofv3 --marker-trace --kernel-trace` timelines next to the kernels they enqueue.
// Cost when no profiler is attached: one call into an empty roctx stub.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace mx {

class TraceRange {
   public:
    explicit TraceRange(const char* name) { roctxRangePushA(name); }
    ~TraceRange() { roctxRangePop(); }
    TraceRange(const TraceRange&) = delete;
    TraceRange& operator=(const TraceRange&) = delete;
};

inline void trace_mark(const char* name) { roctxMarkA(name); }

}  // namespace mx
