// roctx ranges around the data-plane stages, so `rocprofv3 --marker-trace
// --kernel-trace --memory-copy-trace` shows each read, each ring-slot hand-off
// (H2D copy + CRC launches being enqueued) and each wait for landed bytes on
// the same timeline as the SDMA copies and the CRC kernels.  [new]
// ("roctx ranges around ring-slot H2D/CRC stages").
// Without a profiler attached a range is a cheap call into the roctx stub.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace gcsb {

class RoctxRange {
 public:
  explicit RoctxRange(const char* name) { roctxRangePushA(name); }
  ~RoctxRange() { roctxRangePop(); }
  RoctxRange(const RoctxRange&) = delete;
  RoctxRange& operator=(const RoctxRange&) = delete;
};

}  // namespace gcsb
