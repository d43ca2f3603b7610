// Can the receiving core land bytes straight in HBM through the PCIe BAR?
//
// Every read today is recv() into a pinned host ring, then an SDMA copy to
// HBM. If the GPU's VRAM is CPU-mapped (large BAR) the receive could write
// HBM directly: no ring, no H2D copy, and the CPU's stores into
// write-combined VRAM carry no read-for-ownership of the destination.
// This probe measures, on one MI355X:
//   - whether the device is large-BAR and fine-grained VRAM is host-mapped;
//   - one core's memcpy DRAM -> DRAM (THP) vs DRAM -> VRAM (fine-grained);
//   - one loopback TCP stream (sendfile of a memfd) recv()'d into DRAM (THP)
//     vs into VRAM, with the receiving thread's CPU time;
//   - that the bytes written through the BAR are what the GPU sees.
// Build: hipcc --offload-arch=gfx950 -O2 -o bar_probe bar_probe.hip
// Output: one JSON line.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <setjmp.h>
#include <signal.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double thread_cpu_s() {
  rusage ru{};
  getrusage(RUSAGE_THREAD, &ru);
  return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));        \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

static sigjmp_buf g_jmp;
static void on_segv(int) { siglongjmp(g_jmp, 1); }

// Does a CPU store to p fault?  (A SIGSEGV here is the CPU's own page fault on
// an address with no host mapping; the GPU is not involved.)
static bool cpu_writable(void* p) {
  struct sigaction sa{}, old{};
  sa.sa_handler = on_segv;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &old);
  sigaction(SIGBUS, &sa, nullptr);
  bool ok = false;
  if (sigsetjmp(g_jmp, 1) == 0) {
    *static_cast<volatile uint32_t*>(p) = 0x12345678u;
    ok = true;
  }
  sigaction(SIGSEGV, &old, nullptr);
  signal(SIGBUS, SIG_DFL);
  return ok;
}

static void* thp_alloc(size_t n) {
  void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return nullptr;
  madvise(p, n, MADV_HUGEPAGE);
  std::memset(p, 0, n);
  return p;
}

// one loopback TCP stream: sender thread sendfile()s `total` bytes of a memfd
// in 16 MiB pieces; the calling thread recv()s into dst (a ring of ring_bytes).
// Returns GB/s; *cpu = receiving thread CPU-s per GiB.
static double tcp_into(uint8_t* dst, size_t ring_bytes, size_t total, int memfd, double* cpu) {
  int ls = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof(a));
  socklen_t al = sizeof(a);
  getsockname(ls, reinterpret_cast<sockaddr*>(&a), &al);
  listen(ls, 1);
  std::thread snd([&] {
    int s = accept(ls, nullptr, nullptr);
    size_t left = total;
    off_t off = 0;
    const size_t fsz = 256u << 20;
    while (left) {
      size_t k = left < (16u << 20) ? left : (16u << 20);
      if (static_cast<size_t>(off) + k > fsz) off = 0;
      ssize_t w = sendfile(s, memfd, &off, k);
      if (w <= 0) break;
      left -= static_cast<size_t>(w);
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
    size_t want = ring_bytes - pos;
    if (want > (4u << 20)) want = 4u << 20;
    ssize_t r = recv(c, dst + pos, want, 0);
    if (r <= 0) break;
    got += static_cast<size_t>(r);
    pos = (pos + static_cast<size_t>(r)) % ring_bytes;
  }
  const double el = now_s() - t0;
  *cpu = (thread_cpu_s() - c0) / (static_cast<double>(got) / (1u << 30));
  close(c);
  snd.join();
  close(ls);
  return got / el / 1e9;
}

int main() {
  CHECK(hipSetDevice(0));
  int large = 0;
  CHECK(hipDeviceGetAttribute(&large, hipDeviceAttributeIsLargeBar, 0));
  const size_t N = 256u << 20, RING = 16u << 20;
  std::string out = "{\"large_bar\": " + std::to_string(large);

  // fine-grained VRAM and its host mapping
  void* vram = nullptr;
  hipError_t e = hipExtMallocWithFlags(&vram, N, hipDeviceMallocFinegrained);
  if (e != hipSuccess) {
    std::printf("%s, \"error\": \"hipExtMallocWithFlags: %s\"}\n", out.c_str(), hipGetErrorString(e));
    return 0;
  }
  hipPointerAttribute_t attr{};
  CHECK(hipPointerGetAttributes(&attr, vram));
  hsa_amd_pointer_info_t pi{};
  pi.size = sizeof(pi);
  const hsa_status_t hs = hsa_amd_pointer_info(vram, &pi, nullptr, nullptr, nullptr);
  char b[384];
  std::snprintf(b, sizeof(b),
                ", \"hip_host_pointer\": %s, \"hsa_status\": %d, \"hsa_type\": %d, \"hsa_host_base\": %s, "
                "\"hsa_agent_base_is_ptr\": %s",
                attr.hostPointer ? "true" : "false", static_cast<int>(hs), static_cast<int>(pi.type),
                pi.hostBaseAddress ? "true" : "false", pi.agentBaseAddress == vram ? "true" : "false");
  out += b;
  uint8_t* hv = static_cast<uint8_t*>(attr.hostPointer ? attr.hostPointer
                                      : (pi.hostBaseAddress ? pi.hostBaseAddress : vram));
  const bool host_ok = cpu_writable(hv);
  std::snprintf(b, sizeof(b), ", \"cpu_store_ok\": %s", host_ok ? "true" : "false");
  out += b;
  if (!host_ok) {
    std::printf("%s}\n", out.c_str());
    return 0;
  }

  uint8_t* src = static_cast<uint8_t*>(thp_alloc(N));
  uint8_t* dram = static_cast<uint8_t*>(thp_alloc(N));
  for (size_t i = 0; i < N; i += 8) *reinterpret_cast<uint64_t*>(src + i) = i * 0x9E3779B97F4A7C15ull;

  // one core's memcpy, 3 passes each, best
  auto best_copy = [&](uint8_t* dst) {
    double best = 0;
    for (int k = 0; k < 3; ++k) {
      const double t0 = now_s();
      std::memcpy(dst, src, N);
      const double g = N / (now_s() - t0) / 1e9;
      if (g > best) best = g;
    }
    return best;
  };
  const double mc_dram = best_copy(dram);
  const double mc_vram = best_copy(hv);
  // the GPU sees what the CPU wrote through the BAR
  std::vector<uint8_t> back(4096);
  bool ok = true;
  for (size_t off : {size_t(0), N / 2 + 12345, N - 4096}) {
    CHECK(hipMemcpy(back.data(), static_cast<uint8_t*>(vram) + off, 4096, hipMemcpyDeviceToHost));
    if (std::memcmp(back.data(), src + off, 4096) != 0) ok = false;
  }
  std::snprintf(b, sizeof(b), ", \"memcpy_dram_gbps\": %.2f, \"memcpy_vram_gbps\": %.2f, \"vram_bytes_match\": %s",
                mc_dram, mc_vram, ok ? "true" : "false");
  out += b;

  // loopback TCP: 2 GiB into a 16 MiB ring in DRAM, then in VRAM, twice each
  int mfd = memfd_create("bar_probe", 0);
  if (ftruncate(mfd, N) != 0) return 1;
  void* mp = mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_SHARED, mfd, 0);
  std::memcpy(mp, src, N);
  munmap(mp, N);
  for (int rep = 0; rep < 2; ++rep) {
    double cd = 0, cv = 0;
    const double gd = tcp_into(dram, RING, 2ull << 30, mfd, &cd);
    const double gv = tcp_into(hv, RING, 2ull << 30, mfd, &cv);
    std::snprintf(b, sizeof(b),
                  ", \"tcp_dram_gbps_%d\": %.2f, \"tcp_dram_cpu_s_per_gib_%d\": %.4f, \"tcp_vram_gbps_%d\": %.2f, "
                  "\"tcp_vram_cpu_s_per_gib_%d\": %.4f",
                  rep, gd, rep, cd, rep, gv, rep, cv);
    out += b;
  }
  std::printf("%s}\n", out.c_str());
  (void)hipFree(vram);
  return 0;
}
