// loopback_ceiling: how fast can ONE core move an object's bytes off one
// loopback TCP stream into a host ring?  No GPU, no HTTP/2, no gRPC framing.
//
// The headline bench reads a 256 MiB object over ONE gRPC stream (the
// reference's one NewReader per read, reference main.go:134-140).  On one TCP
// connection every byte is copied out of the socket by one receiving thread,
// so that thread's copy rate bounds the read.  This tool measures that bound
// on the same box, in the same placement, with the pieces taken away one by
// one:
//   memcpy  one thread copying a DRAM-resident object into the ring (the
//           kernel's copy_to_user does the same work for recv());
//   tcp     the object in a memfd, sendfile()d by a sender thread over a
//           loopback connection, recv()d by a receiver thread into the ring
//           (exactly the endpoint/client split of the bench, minus framing).
// Reports GB/s and CPU-seconds per GiB of each thread (RUSAGE_THREAD).
//
//   loopback_ceiling [--mode tcp|memcpy|both] [--object-mib 256] [--reads 10]
//                    [--ring-kib 16384] [--recv-kib 4096] [--rcvbuf-kib 0]
//                    [--send-cpu N] [--recv-cpu N] [--zerocopy-send 1] [--ring-pages 0|1|2]
//
// The measurement itself lives in core/ceiling.cc (bench.py's `ceiling`
// block runs the same code in the headline's placement).
#include <cstdio>
#include <exception>
#include <string>

#include "core/ceiling.h"
#include "tools/goflags.h"

int main(int argc, char** argv) {
  gcsb::GoFlags fs("loopback_ceiling");
  auto* mode = fs.String("mode", "both", "tcp | memcpy | both");
  auto* obj_mib = fs.Int("object-mib", 256, "object size (MiB)");
  auto* reads = fs.Int("reads", 10, "timed reads");
  auto* ring_kib = fs.Int("ring-kib", 16384, "receive ring size (KiB); 16 MiB = the bench's 4x4 MiB ring");
  auto* recv_kib = fs.Int("recv-kib", 4096, "bytes asked per recv() (KiB)");
  auto* rcvbuf_kib = fs.Int("rcvbuf-kib", 0, "SO_RCVBUF (KiB), 0 = autotuning");
  auto* send_cpu = fs.Int("send-cpu", -1, "pin the sender to this CPU (-1 = unpinned)");
  auto* recv_cpu = fs.Int("recv-cpu", -1, "pin the receiver to this CPU (-1 = unpinned)");
  auto* zc = fs.Bool("zerocopy-send", true, "sender sends zero-copy (the endpoint's path)");
  auto* thp = fs.Bool("thp-source", true, "zero-copy from THP memory by vmsplice (the endpoint's default); "
                      "false = sendfile() from a memfd");
  auto* pages = fs.Int("ring-pages", 0, "ring pages: 0 system default, 1 huge (MADV_HUGEPAGE), 2 small");
  fs.Parse(argc, argv);
  gcsb::CeilingConfig c;
  c.object_bytes = static_cast<size_t>(*obj_mib) << 20;
  c.reads = static_cast<int>(*reads);
  c.ring_bytes = static_cast<size_t>(*ring_kib) << 10;
  c.recv_chunk = static_cast<size_t>(*recv_kib) << 10;
  c.rcvbuf = static_cast<int>(*rcvbuf_kib) << 10;
  if (*send_cpu >= 0) c.send_cpus = {static_cast<int>(*send_cpu)};
  if (*recv_cpu >= 0) c.recv_cpus = {static_cast<int>(*recv_cpu)};
  c.zerocopy_send = *zc;
  c.thp_source = *thp;
  c.ring_pages = static_cast<int>(*pages);
  std::printf("{\"object_mib\": %lld, \"reads\": %lld, \"ring_kib\": %lld, \"recv_kib\": %lld",
              static_cast<long long>(*obj_mib), static_cast<long long>(*reads), static_cast<long long>(*ring_kib),
              static_cast<long long>(*recv_kib));
  try {
    if (*mode == "memcpy" || *mode == "both") {
      gcsb::CeilingResult m = gcsb::memcpy_ceiling(c);
      std::printf(", \"memcpy_gbps\": %.2f, \"memcpy_cpu_s_per_gib\": %.4f", m.gbps, m.recv_cpu_s_per_gib);
    }
    if (*mode == "tcp" || *mode == "both") {
      gcsb::CeilingResult t = gcsb::tcp_ceiling(c);
      std::printf(", \"tcp_gbps\": %.2f, \"tcp_p50_ms\": %.3f, \"recv_cpu_s_per_gib\": %.4f, "
                  "\"send_cpu_s_per_gib\": %.4f",
                  t.gbps, t.p50_ms, t.recv_cpu_s_per_gib, t.send_cpu_s_per_gib);
    }
  } catch (const std::exception& e) {
    std::printf("}\n");
    std::fprintf(stderr, "loopback_ceiling: %s\n", e.what());
    return 1;
  }
  std::printf("}\n");
  return 0;
}
