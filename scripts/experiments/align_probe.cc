// Does the receive copy care about the source's alignment?
//
// The synthetic endpoint sendfile()s object bytes from a memfd at the
// object's rotation offset, which is any byte offset: the skb fragments the
// receiver copies from then start at arbitrary addresses while the ring slot
// it copies into is page-aligned.  This probe measures one core:
//   - `rep movsb` (what copy_to_user uses on FSRM CPUs) of 1 MiB blocks from
//     a source at offset k into a page-aligned destination, k = 0, 8, 13, 64;
//   - one loopback TCP stream, sendfile() of a memfd from file offset k, into
//     a 16 MiB ring (receiver GB/s and CPU-s/GiB).
// Build: g++ -O2 -std=c++17 -pthread -o align_probe align_probe.cc
// Output: one JSON line.
#include <netinet/in.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double thread_cpu_s() {
  rusage ru{};
  getrusage(RUSAGE_THREAD, &ru);
  return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}
static void* thp_alloc(size_t n) {
  void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  madvise(p, n, MADV_HUGEPAGE);
  std::memset(p, 1, n);
  return p;
}
static inline void movsb(void* d, const void* s, size_t n) {
  asm volatile("rep movsb" : "+D"(d), "+S"(s), "+c"(n) : : "memory");
}

// src: 256 MiB (cold across passes); dst: 16 MiB ring
static double movsb_gbps(const uint8_t* src, uint8_t* dst, size_t k) {
  const size_t blk = 1u << 20, total = 256u << 20, ring = 16u << 20;
  double best = 0;
  for (int rep = 0; rep < 3; ++rep) {
    const double t0 = now_s();
    size_t pos = 0;
    for (size_t off = 0; off + blk + 64 <= total; off += blk) {
      movsb(dst + pos, src + off + k, blk);
      pos = (pos + blk) % ring;
    }
    const double g = (total - blk) / (now_s() - t0) / 1e9;
    if (g > best) best = g;
  }
  return best;
}

static double tcp_gbps(int memfd, size_t k, uint8_t* dst, double* cpu) {
  const size_t total = 2ull << 30, ring = 16u << 20, fsz = 256u << 20;
  int ls = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof(a));
  socklen_t al = sizeof(a);
  getsockname(ls, reinterpret_cast<sockaddr*>(&a), &al);
  listen(ls, 1);
  std::thread snd([&] {
    int s = accept(ls, nullptr, nullptr);
    size_t left = total;
    while (left) {
      off_t off = static_cast<off_t>(k);
      size_t chunk = fsz - (1u << 20);  // from offset k, whole-file passes
      if (chunk > left) chunk = left;
      while (chunk) {
        ssize_t w = sendfile(s, memfd, &off, chunk);
        if (w <= 0) break;
        chunk -= static_cast<size_t>(w);
        left -= static_cast<size_t>(w);
      }
    }
    close(s);
  });
  int c = socket(AF_INET, SOCK_STREAM, 0);
  int rb = 64 << 20;
  setsockopt(c, SOL_SOCKET, SO_RCVBUF, &rb, sizeof(rb));
  connect(c, reinterpret_cast<sockaddr*>(&a), sizeof(a));
  size_t got = 0, pos = 0;
  const double c0 = thread_cpu_s(), t0 = now_s();
  while (got < total) {
    size_t want = ring - pos;
    if (want > (2u << 20)) want = 2u << 20;
    ssize_t r = recv(c, dst + pos, want, 0);
    if (r <= 0) break;
    got += static_cast<size_t>(r);
    pos = (pos + static_cast<size_t>(r)) % ring;
  }
  const double el = now_s() - t0;
  *cpu = (thread_cpu_s() - c0) / (got / double(1u << 30));
  close(c);
  snd.join();
  close(ls);
  return got / el / 1e9;
}

int main() {
  uint8_t* src = static_cast<uint8_t*>(thp_alloc(256u << 20));
  uint8_t* dst = static_cast<uint8_t*>(thp_alloc(16u << 20));
  std::string out = "{";
  char b[160];
  for (size_t k : {0, 8, 13, 64}) {
    std::snprintf(b, sizeof(b), "%s\"movsb_src_off_%zu_gbps\": %.2f", out.size() > 1 ? ", " : "", k,
                  movsb_gbps(src, dst, k));
    out += b;
  }
  int mfd = memfd_create("align_probe", 0);
  if (ftruncate(mfd, 256u << 20) != 0) return 1;
  void* mp = mmap(nullptr, 256u << 20, PROT_READ | PROT_WRITE, MAP_SHARED, mfd, 0);
  std::memcpy(mp, src, 256u << 20);
  munmap(mp, 256u << 20);
  for (int rep = 0; rep < 2; ++rep)
    for (size_t k : {0, 13}) {
      double cpu = 0;
      const double g = tcp_gbps(mfd, k, dst, &cpu);
      std::snprintf(b, sizeof(b), ", \"tcp_off_%zu_gbps_%d\": %.2f, \"tcp_off_%zu_cpu_s_per_gib_%d\": %.4f", k, rep,
                    g, k, rep, cpu);
      out += b;
    }
  std::printf("%s}\n", out.c_str());
  return 0;
}
