// Page-cache-friendly receive destinations: 2 MiB-aligned anonymous memory
// with MADV_HUGEPAGE, faulted in at allocation.
//
// Every object byte a socket delivers is written by the kernel's
// copy_to_user into a destination like these.  Into the GPU sink's THP ring
// one receiving core moves ~19-20 GB/s (0.05 CPU-s/GiB); the same copy into
// 4 KiB-page heap blocks cost 0.09 CPU-s/GiB (profiles/r3_mux:
// gcsb-h2-reader of the 48-worker discard-sink reads), a TLB miss every 4 KiB
// of a 2 MiB message.  The discard sinks, the endpoint's upload receive
// buffers and the CRC bench buffers use these.
#pragma once
#include <cstddef>
#include <cstdint>

namespace gcsb {

// n bytes (rounded up to 2 MiB), 2 MiB-aligned, THP-advised, pre-faulted;
// throws std::bad_alloc.  Free with huge_free(p, n) (same n).
uint8_t* huge_alloc(size_t n);
void huge_free(void* p, size_t n);

// Process-wide LIFO pool of huge_alloc() buffers by rounded size: the buffer
// handed out is the one handed back most recently (cache-warm), and nothing
// is mapped / unmapped per request once the pool is warm.  Mapping and
// faulting a fresh THP buffer per request cost the endpoint's connection
// thread 0.1 CPU-s/GiB on 1 MiB reads and stalled neighbours in compaction
// (profiles/r3_b).  Holds at most 1 GiB; beyond that buffers are unmapped.
uint8_t* huge_take(size_t n);
void huge_give(void* p, size_t n);

// Bytes of [p, p+len) the kernel backs with transparent huge pages
// (/proc/self/smaps AnonHugePages of the VMAs overlapping the range, capped
// at len): MADV_HUGEPAGE is advice, and on a fragmented host the ring can
// silently fall back to 4 KiB pages.  -1 if smaps is unreadable.
long long thp_bytes_of(const void* p, size_t len);
inline size_t huge_round(size_t n) { return (n + (size_t(2) << 20) - 1) / (size_t(2) << 20) * (size_t(2) << 20); }

// Owning, movable huge_alloc() buffer.
class HugeBuffer {
 public:
  HugeBuffer() = default;
  explicit HugeBuffer(size_t n) : p_(huge_take(n)), cap_(huge_round(n)) {}
  ~HugeBuffer() { huge_give(p_, cap_); }
  HugeBuffer(HugeBuffer&& o) noexcept : p_(o.p_), cap_(o.cap_) { o.p_ = nullptr, o.cap_ = 0; }
  HugeBuffer& operator=(HugeBuffer&& o) noexcept {
    if (this != &o) {
      huge_give(p_, cap_);
      p_ = o.p_, cap_ = o.cap_;
      o.p_ = nullptr, o.cap_ = 0;
    }
    return *this;
  }
  HugeBuffer(const HugeBuffer&) = delete;
  HugeBuffer& operator=(const HugeBuffer&) = delete;
  char* get() const { return reinterpret_cast<char*>(p_); }
  size_t capacity() const { return cap_; }
  explicit operator bool() const { return p_ != nullptr; }

 private:
  uint8_t* p_ = nullptr;
  size_t cap_ = 0;
};

}  // namespace gcsb
