// Same-box ceilings for the one-stream read: how fast can ONE receiving core
// move an object's bytes off one loopback TCP stream into a host ring, with
// no GPU, no HTTP/2 and no gRPC framing (and the plain memcpy rate of that
// core for comparison).  Used by tools/loopback_ceiling and by bench.py's
// `ceiling` block, which runs it in the headline's own placement so the
// headline can be read as a fraction of its bound.
//
// The headline reads a 256 MiB object over ONE gRPC stream (the reference's
// one NewReader per read, reference main.go:134-140); on one TCP connection
// every byte is copied out of the socket by one thread, so that thread's
// copy_to_user rate bounds the read.
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace gcsb {

struct CeilingResult {
  double gbps = 0;                 // bytes moved / wall time (1e9 B/s)
  double p50_ms = 0;               // per object
  double recv_cpu_s_per_gib = 0;   // receiving (or copying) thread
  double send_cpu_s_per_gib = 0;   // sending thread (tcp)
};

// The sender's bytes for tcp_ceiling's upload bound: one object per read,
// sent by reference (vmsplice + splice) and left unchanged until end(), which
// runs once the receiver holds every byte.  bindings.cc wraps the uploader's
// own GpuByteSource (HBM staged into pinned slots by D2H copies), so the probe
// sends the pages a timed upload sends, written the way it writes them.
class CeilingSource {
 public:
  virtual ~CeilingSource() = default;
  virtual void begin() = 0;
  virtual std::pair<const uint8_t*, size_t> next(size_t max) = 0;
  virtual void end() = 0;
};

struct CeilingConfig {
  size_t object_bytes = size_t(256) << 20;
  int reads = 10;
  size_t ring_bytes = size_t(16) << 20;   // receive ring (the bench's 8 x 2 MiB)
  size_t recv_chunk = size_t(4) << 20;    // bytes asked per recv()
  int rcvbuf = 0;                         // SO_RCVBUF, 0 = autotuning
  std::vector<int> send_cpus, recv_cpus;  // empty = unpinned
  bool zerocopy_send = true;              // zero-copy send, from the endpoint's source:
  // THP anonymous memory by vmsplice + splice (PatternBuffer::send_by_vmsplice,
  // the endpoint's default) or a memfd by sendfile
  bool thp_source = true;
  int ring_pages = 1;                     // 0 default, 1 MADV_HUGEPAGE (the THP ring), 2 small pages
  CeilingSource* source = nullptr;        // tcp: the sender's bytes (default: the object above)
};

// One thread memcpy()s a DRAM-resident object into the ring (recv_cpus).
CeilingResult memcpy_ceiling(const CeilingConfig& c);
// A sender thread sends an object (zero-copy, as the endpoint does) over one
// loopback connection, a receiver thread recv()s it into the ring.  Throws
// std::runtime_error.
CeilingResult tcp_ceiling(const CeilingConfig& c);

}  // namespace gcsb
