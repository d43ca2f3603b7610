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
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "core/affinity.h"
#include "tools/goflags.h"

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double thread_cpu_s() {
  rusage ru{};
  getrusage(RUSAGE_THREAD, &ru);
  return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}

void pin(int cpu) {
  if (cpu >= 0) gcsb::pin_current_thread({cpu});
}

[[noreturn]] void die(const char* what) {
  std::perror(what);
  std::exit(1);
}

struct Result {
  double gbps = 0, recv_cpu_per_gib = 0, send_cpu_per_gib = 0, p50_ms = 0;
};

// ring pages: 0 = system default, 1 = MADV_HUGEPAGE, 2 = MADV_NOHUGEPAGE
int g_ring_pages = 0;

uint8_t* alloc_ring(size_t n) {
  void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) die("mmap(ring)");
  if (g_ring_pages == 1) (void)madvise(p, n, MADV_HUGEPAGE);
  if (g_ring_pages == 2) (void)madvise(p, n, MADV_NOHUGEPAGE);
  (void)mlock(p, n);  // page-locked like the pinned ring when allowed
  std::memset(p, 0, n);
  return static_cast<uint8_t*>(p);
}

Result run_memcpy(size_t obj, int reads, size_t ring, int pin_cpu) {
  pin(pin_cpu);
  std::vector<uint8_t> src(obj);
  for (size_t i = 0; i < obj; i += 4096) src[i] = static_cast<uint8_t>(i >> 12);
  uint8_t* dst = alloc_ring(ring);
  const size_t piece = std::min<size_t>(ring, 2u << 20);
  std::vector<double> lat;
  double c0 = thread_cpu_s(), t0 = now_s();
  for (int r = 0; r < reads; ++r) {
    double a = now_s();
    size_t off = 0, roff = 0;
    while (off < obj) {
      size_t k = std::min(piece, obj - off);
      if (roff + k > ring) roff = 0;
      std::memcpy(dst + roff, src.data() + off, k);
      off += k;
      roff += k;
    }
    lat.push_back((now_s() - a) * 1e3);
  }
  double el = now_s() - t0, cpu = thread_cpu_s() - c0;
  munmap(dst, ring);
  std::sort(lat.begin(), lat.end());
  Result res;
  res.gbps = static_cast<double>(obj) * reads / el / 1e9;
  res.recv_cpu_per_gib = cpu / (static_cast<double>(obj) * reads / (1 << 30));
  res.p50_ms = lat[lat.size() / 2];
  return res;
}

Result run_tcp(size_t obj, int reads, size_t ring, size_t recv_chunk, int rcvbuf, int send_cpu, int recv_cpu,
               bool zerocopy_send) {
  int mfd = memfd_create("ceiling-object", 0);
  if (mfd < 0) die("memfd_create");
  if (ftruncate(mfd, static_cast<off_t>(obj)) != 0) die("ftruncate");
  {
    std::vector<uint8_t> blk(1 << 20);
    for (size_t i = 0; i < blk.size(); ++i) blk[i] = static_cast<uint8_t>(i * 131 + 7);
    for (size_t off = 0; off < obj; off += blk.size())
      if (pwrite(mfd, blk.data(), std::min(blk.size(), obj - off), static_cast<off_t>(off)) < 0) die("pwrite");
  }
  int ls = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || listen(ls, 1) != 0) die("bind/listen");
  socklen_t al = sizeof(a);
  getsockname(ls, reinterpret_cast<sockaddr*>(&a), &al);
  std::atomic<int> go{0};
  std::atomic<bool> quit{false};
  double send_cpu_total = 0;
  std::thread sender([&] {
    gcsb::name_current_thread("ceiling-send");
    pin(send_cpu);
    int s = accept(ls, nullptr, nullptr);
    if (s < 0) die("accept");
    int one = 1;
    setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::vector<uint8_t> copybuf;
    if (!zerocopy_send) copybuf.resize(2u << 20);
    double c0 = thread_cpu_s();
    for (int r = 0; r < reads; ++r) {
      while (go.load() <= r && !quit.load()) std::this_thread::yield();
      if (quit.load()) break;
      off_t off = 0;
      while (static_cast<size_t>(off) < obj) {
        size_t k = std::min<size_t>(obj - off, 2u << 20);
        if (zerocopy_send) {
          ssize_t w = sendfile(s, mfd, &off, k);
          if (w <= 0) die("sendfile");
        } else {
          if (pread(mfd, copybuf.data(), k, off) != static_cast<ssize_t>(k)) die("pread");
          size_t done = 0;
          while (done < k) {
            ssize_t w = send(s, copybuf.data() + done, k - done, 0);
            if (w <= 0) die("send");
            done += static_cast<size_t>(w);
          }
          off += static_cast<off_t>(k);
        }
      }
    }
    send_cpu_total = thread_cpu_s() - c0;
    close(s);
  });
  Result res;
  std::thread receiver([&] {
    gcsb::name_current_thread("ceiling-recv");
    pin(recv_cpu);
    int c = socket(AF_INET, SOCK_STREAM, 0);
    if (rcvbuf > 0) setsockopt(c, SOL_SOCKET, SO_RCVBUF, &rcvbuf, sizeof(rcvbuf));
    if (connect(c, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) die("connect");
    uint8_t* dst = alloc_ring(ring);
    std::vector<double> lat;
    double c0 = thread_cpu_s(), t0 = now_s();
    for (int r = 0; r < reads; ++r) {
      double st = now_s();
      go.store(r + 1);
      size_t got = 0, roff = 0;
      while (got < obj) {
        if (roff >= ring) roff = 0;
        size_t want = std::min({recv_chunk, ring - roff, obj - got});
        ssize_t n = recv(c, dst + roff, want, 0);
        if (n <= 0) die("recv");
        got += static_cast<size_t>(n);
        roff += static_cast<size_t>(n);
      }
      lat.push_back((now_s() - st) * 1e3);
    }
    double el = now_s() - t0, cpu = thread_cpu_s() - c0;
    std::sort(lat.begin(), lat.end());
    res.gbps = static_cast<double>(obj) * reads / el / 1e9;
    res.recv_cpu_per_gib = cpu / (static_cast<double>(obj) * reads / (1 << 30));
    res.p50_ms = lat[lat.size() / 2];
    munmap(dst, ring);
    close(c);
  });
  receiver.join();
  quit.store(true);
  sender.join();
  res.send_cpu_per_gib = send_cpu_total / (static_cast<double>(obj) * reads / (1 << 30));
  close(ls);
  close(mfd);
  return res;
}

}  // namespace

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
  auto* zc = fs.Bool("zerocopy-send", true, "sender uses sendfile() (the endpoint's path)");
  auto* pages = fs.Int("ring-pages", 0, "ring pages: 0 system default, 1 huge (MADV_HUGEPAGE), 2 small");
  fs.Parse(argc, argv);
  g_ring_pages = static_cast<int>(*pages);
  const size_t obj = static_cast<size_t>(*obj_mib) << 20;
  const size_t ring = static_cast<size_t>(*ring_kib) << 10;
  std::printf("{\"object_mib\": %lld, \"reads\": %lld, \"ring_kib\": %lld, \"recv_kib\": %lld",
              static_cast<long long>(*obj_mib), static_cast<long long>(*reads), static_cast<long long>(*ring_kib),
              static_cast<long long>(*recv_kib));
  if (*mode == "memcpy" || *mode == "both") {
    Result m = run_memcpy(obj, static_cast<int>(*reads), ring, static_cast<int>(*recv_cpu));
    std::printf(", \"memcpy_gbps\": %.2f, \"memcpy_cpu_s_per_gib\": %.4f", m.gbps, m.recv_cpu_per_gib);
  }
  if (*mode == "tcp" || *mode == "both") {
    Result t = run_tcp(obj, static_cast<int>(*reads), ring, static_cast<size_t>(*recv_kib) << 10,
                       static_cast<int>(*rcvbuf_kib) << 10, static_cast<int>(*send_cpu),
                       static_cast<int>(*recv_cpu), *zc);
    std::printf(", \"tcp_gbps\": %.2f, \"tcp_p50_ms\": %.3f, \"recv_cpu_s_per_gib\": %.4f, "
                "\"send_cpu_s_per_gib\": %.4f",
                t.gbps, t.p50_ms, t.recv_cpu_per_gib, t.send_cpu_per_gib);
  }
  std::printf("}\n");
  return 0;
}
