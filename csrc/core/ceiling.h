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
#include <vector>

namespace gcsb {

struct CeilingResult {
  double gbps = 0;                 // bytes moved / wall time (1e9 B/s)
  double p50_ms = 0;               // per object
  double recv_cpu_s_per_gib = 0;   // receiving (or copying) thread
  double send_cpu_s_per_gib = 0;   // sending thread (tcp)
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
};

// One thread memcpy()s a DRAM-resident object into the ring (recv_cpus).
CeilingResult memcpy_ceiling(const CeilingConfig& c);
// A sender thread sends an object (zero-copy, as the endpoint does) over one
// loopback connection, a receiver thread recv()s it into the ring.  Throws
// std::runtime_error.
CeilingResult tcp_ceiling(const CeilingConfig& c);

}  // namespace gcsb
