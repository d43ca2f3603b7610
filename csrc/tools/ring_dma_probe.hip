// ring_dma_probe: does the GPU reading a CPU-written pinned ring slow the
// core that writes it?  (The one-stream headline's receiving core copies
// 5-8% dearer per byte when the copy engine reads its ring than when nothing
// does: profiles/r4_recvcost, r5_window.)  This takes TCP out of it: one
// writer core copies a large DRAM-resident source into a SLOTS x SLOT
// pinned ring slot by slot, as the receive copy does; a submitter core (same
// L3, like the headline's aux core) hands each filled slot to the device;
// the writer reuses a slot once a host-mapped flag says the device is done
// with it (no HIP call on the writer, as in the sink).  A variant is
// WRITER/DEVICE, run interleaved:
//   writer  memcpy  glibc memcpy
//           rep     rep movsb (what the kernel's copy_to_user does)
//           nt      non-temporal stores
//           flush   memcpy, then clflushopt of the slot
//           tcpv / repv  the same into fine-grained VRAM mapped to the host
//                   (large BAR): the receive lands in HBM, nothing to copy
//           tcp     recv() from one loopback TCP connection whose sender
//                   (sender=CPU) vmsplice()s the source into the socket, as
//                   the endpoint does: the headline minus HTTP/2 and gRPC
//   device  idle    no device work: the submitter sets the flag itself
//           flag    a one-thread kernel writes the flag (HIP launch only)
//           sdma    hipMemcpyAsync H2D of the slot into HBM, then the flag
//                   kernel (the headline's path)
//           kernel  a GPU kernel pulls the slot over the host link into
//                   HBM, then the flag kernel
//           sdma_clwb / sdma_flush  the submitter clwb's / clflushopt's the
//                   slot before its H2D copy
//           relay   the submitter copies the slot (rep movsb) into
//                   host-mapped fine-grained VRAM itself: no device read
//           relaynt the same with non-temporal stores
//           sdma_pw the submitter prefetchw's the slot after its H2D copy
//                   finished, before handing it back to the writer
//
//   ring_dma_probe slots=4 slot=1048576 total=2147483648 reps=5 \
//                  writer=8 submitter=9 variants=memcpy/idle,memcpy/sdma,rep/sdma
// One JSON line per (rep, variant): writer GB/s, the writer's wait for slots.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sched.h>
#include <setjmp.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cctype>
#include <cstdio>
#include <fstream>
#include <cstdlib>
#include <cstring>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
    std::exit(2);
  }
}

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

int64_t thread_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

void pin(int cpu) {
  if (cpu < 0) return;
  cpu_set_t s;
  CPU_ZERO(&s);
  CPU_SET(cpu, &s);
  sched_setaffinity(0, sizeof(s), &s);
}

__global__ void flag_kernel(volatile uint32_t* flag, uint32_t v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    __threadfence_system();
    *flag = v;
  }
}

// host slot -> HBM, 16 B per lane per step; grid-stride
__global__ void pull_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}

void rep_movsb(uint8_t* dst, const uint8_t* src, size_t n) {
  asm volatile("rep movsb" : "+D"(dst), "+S"(src), "+c"(n) : : "memory");
}

void nt_copy(uint8_t* dst, const uint8_t* src, size_t n) {
  // dst and n are 64-byte multiples here
  for (size_t o = 0; o < n; o += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + o));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + o + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + o + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + o + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o + 48), d);
  }
  _mm_sfence();
}

__attribute__((target("clwb"))) void clwb_range(const uint8_t* p, size_t n) {
  for (size_t o = 0; o < n; o += 64) _mm_clwb(const_cast<uint8_t*>(p + o));
  _mm_sfence();
}

__attribute__((target("clflushopt"))) void flush_range(const uint8_t* p, size_t n) {
  for (size_t o = 0; o < n; o += 64) _mm_clflushopt(const_cast<uint8_t*>(p + o));
  _mm_sfence();
}

// Interrupts taken by `cpus` since boot, by source (/proc/interrupts: the
// first line names the CPU of each column; the source is the line's label
// plus, for device lines, the last field).
std::map<std::string, uint64_t> irqs_on(const std::vector<int>& cpus) {
  std::map<std::string, uint64_t> out;
  std::ifstream f("/proc/interrupts");
  std::string line;
  if (!std::getline(f, line)) return out;
  std::vector<int> col_cpu;
  {
    std::stringstream hs(line);
    std::string t;
    while (hs >> t)
      if (t.rfind("CPU", 0) == 0) col_cpu.push_back(std::atoi(t.c_str() + 3));
  }
  while (std::getline(f, line)) {
    std::stringstream ls(line);
    std::string label;
    ls >> label;
    std::vector<uint64_t> v;
    std::string t;
    std::string rest;
    for (size_t c = 0; c < col_cpu.size() && ls >> t; ++c) {
      if (t.empty() || !std::isdigit(static_cast<unsigned char>(t[0]))) {
        rest = t;
        break;
      }
      v.push_back(std::strtoull(t.c_str(), nullptr, 10));
    }
    std::string last = rest;
    while (ls >> t) last = t;
    const std::string key = label + (last.empty() ? "" : " " + last);
    for (size_t c = 0; c < v.size(); ++c)
      for (int cpu : cpus)
        if (col_cpu[c] == cpu && v[c]) out[key] += v[c];
  }
  return out;
}

int sibling_of(int cpu) {
  std::ifstream f("/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/topology/thread_siblings_list");
  std::string s;
  if (!std::getline(f, s)) return -1;
  std::stringstream ss(s);
  std::string t;
  while (std::getline(ss, t, ',')) {
    const size_t d = t.find('-');
    const int a = std::atoi(t.c_str()), b = d == std::string::npos ? a : std::atoi(t.c_str() + d + 1);
    for (int c = a; c <= b; ++c)
      if (c != cpu) return c;
  }
  return -1;
}

sigjmp_buf g_probe_jmp;
void on_probe_fault(int) { siglongjmp(g_probe_jmp, 1); }

// Whether the CPU can store to p (a device allocation mapped to the host?):
// one store under a SIGSEGV/SIGBUS handler.
bool host_writable(volatile uint8_t* p) {
  struct sigaction sa {}, old_segv{}, old_bus{};
  sa.sa_handler = on_probe_fault;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &old_segv);
  sigaction(SIGBUS, &sa, &old_bus);
  bool ok = false;
  if (sigsetjmp(g_probe_jmp, 1) == 0) {
    p[0] = 1;
    ok = p[0] == 1;
  }
  sigaction(SIGSEGV, &old_segv, nullptr);
  sigaction(SIGBUS, &old_bus, nullptr);
  return ok;
}

struct Args {
  int slots = 4;
  size_t slot = 1 << 20;
  size_t total = 4ull << 30;
  size_t src_bytes = 512ull << 20;
  int reps = 5;
  int writer = -1, submitter = -1, sender = -1;
  int lag = 0;  // the submitter issues slot seq only once seq + lag was posted (lines age out of the L3 first)
  std::vector<int> rt;  // CPUs for the HIP runtime's own threads (inherited from main at init); empty = as started
  std::vector<std::string> variants{"memcpy/idle", "memcpy/flag", "memcpy/sdma", "rep/idle", "rep/sdma", "nt/sdma"};
};

Args parse(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    const size_t eq = s.find('=');
    if (eq == std::string::npos) continue;
    const std::string k = s.substr(0, eq), v = s.substr(eq + 1);
    if (k == "slots") a.slots = std::atoi(v.c_str());
    else if (k == "slot") a.slot = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "total") a.total = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "src") a.src_bytes = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "reps") a.reps = std::atoi(v.c_str());
    else if (k == "writer") a.writer = std::atoi(v.c_str());
    else if (k == "submitter") a.submitter = std::atoi(v.c_str());
    else if (k == "sender") a.sender = std::atoi(v.c_str());
    else if (k == "lag") a.lag = std::atoi(v.c_str());
    else if (k == "rt") {
      std::stringstream ss(v);
      std::string x;
      while (std::getline(ss, x, ',')) {
        const size_t d = x.find('-');
        const int lo = std::atoi(x.c_str()), hi = d == std::string::npos ? lo : std::atoi(x.c_str() + d + 1);
        for (int c = lo; c <= hi; ++c) a.rt.push_back(c);
      }
    }
    else if (k == "variants") {
      a.variants.clear();
      std::stringstream ss(v);
      std::string x;
      while (std::getline(ss, x, ',')) a.variants.push_back(x);
    }
  }
  return a;
}

}  // namespace

int main(int argc, char** argv) {
  const Args a = parse(argc, argv);
  if (a.slots < 2 || a.slot % 4096 || a.total % a.slot || a.lag < 0 || a.lag >= a.slots) {
    std::fprintf(stderr, "bad geometry\n");
    return 2;
  }
  if (!a.rt.empty()) {
    // the runtime's threads (created during init) inherit this mask; ours re-pin
    cpu_set_t m;
    CPU_ZERO(&m);
    for (int c : a.rt) CPU_SET(c, &m);
    sched_setaffinity(0, sizeof(m), &m);
  }
  check(hipSetDevice(0), "hipSetDevice");
  check(hipFree(nullptr), "hip init");
  // first touch of the source and the ring on the writer's NUMA node (the
  // endpoint builds its send source on its own node, the sink its ring on the
  // receiving thread's): an unpinned main thread put them anywhere, and a
  // remote source cost the receive copy ~25% on one box
  cpu_set_t main_mask;
  CPU_ZERO(&main_mask);
  sched_getaffinity(0, sizeof(main_mask), &main_mask);
  pin(a.writer);
  // the source: THP, faulted in, larger than the L3 (the receive copy's
  // source is the sender's pages, not cache-resident)
  uint8_t* src = static_cast<uint8_t*>(mmap(nullptr, a.src_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS,
                                            -1, 0));
  if (src == MAP_FAILED) return 2;
  madvise(src, a.src_bytes, MADV_HUGEPAGE);
  for (size_t i = 0; i < a.src_bytes; i += 64) src[i] = static_cast<uint8_t>(i * 131);
  uint8_t* ring = nullptr;
  check(hipHostMalloc(reinterpret_cast<void**>(&ring), a.slot * a.slots, hipHostMallocDefault), "hipHostMalloc ring");
  std::memset(ring, 0, a.slot * a.slots);
  sched_setaffinity(0, sizeof(main_mask), &main_mask);
  uint8_t* ring_d = nullptr;
  check(hipHostGetDevicePointer(reinterpret_cast<void**>(&ring_d), ring, 0), "hipHostGetDevicePointer ring");
  uint32_t* flags = nullptr;
  check(hipHostMalloc(reinterpret_cast<void**>(&flags), 64 * a.slots, hipHostMallocMapped | hipHostMallocCoherent),
        "hipHostMalloc flags");
  std::memset(flags, 0, 64 * a.slots);
  uint32_t* flags_d = nullptr;
  check(hipHostGetDevicePointer(reinterpret_cast<void**>(&flags_d), flags, 0), "hipHostGetDevicePointer flags");
  uint8_t* hbm = nullptr;
  check(hipMalloc(reinterpret_cast<void**>(&hbm), a.slot * a.slots * 8), "hipMalloc");
  std::vector<hipStream_t> st(a.slots);
  for (auto& s : st) check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");

  // submitter: a single-slot mailbox per slot (the writer posts seq, the
  // submitter issues the device work for it)
  std::vector<std::atomic<uint64_t>> posted(a.slots);
  for (auto& p : posted) p.store(0);
  std::atomic<int> mode{-1};  // -2: stop
  std::atomic<uint64_t> issued_upto{0};
  std::atomic<uint64_t> last_posted{0};
  std::atomic<bool> draining{false};  // the writer's last slots: no lag
  // device-written completion words for the modes where the submitter
  // post-processes a slot before handing it back (sdma_pw)
  uint32_t* dflags = nullptr;
  check(hipHostMalloc(reinterpret_cast<void**>(&dflags), 64 * a.slots, hipHostMallocMapped | hipHostMallocCoherent),
        "hipHostMalloc dflags");
  std::memset(dflags, 0, 64 * a.slots);
  uint32_t* dflags_d = nullptr;
  check(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflags_d), dflags, 0), "hipHostGetDevicePointer dflags");
  // the relay modes' destination: fine-grained VRAM the host stores to
  uint8_t* vland = nullptr;
  bool vland_ok = false;
  for (const auto& v : a.variants)
    if (v.find("/relay") != std::string::npos) {
      if (hipExtMallocWithFlags(reinterpret_cast<void**>(&vland), a.slot * a.slots * 8, hipDeviceMallocFinegrained) ==
          hipSuccess)
        vland_ok = host_writable(vland);
      std::printf("{\"vram\": \"relay\", \"allocated\": %s, \"host_writable\": %s}\n", vland ? "true" : "false",
                  vland_ok ? "true" : "false");
      std::fflush(stdout);
      break;
    }
  std::thread sub([&] {
    pin(a.submitter);
    uint64_t next = 1;  // the next sequence number to issue (slot (next-1) % slots)
    uint64_t fin = 1;   // sdma_pw: the next sequence number to hand back
    for (;;) {
      const int m = mode.load(std::memory_order_acquire);
      if (m == -2) return;
      if (m == 6 && fin < next) {
        // hand back finished slots in order: take the lines back into this
        // CCD in a writable state first (prefetchw), so the writer's next
        // stores into the slot do not miss to the other side of the fabric
        const int fs = static_cast<int>((fin - 1) % a.slots);
        if (__atomic_load_n(dflags + fs * 16, __ATOMIC_ACQUIRE) == static_cast<uint32_t>(fin)) {
          const uint8_t* p = ring + fs * a.slot;
          for (size_t o = 0; o < a.slot; o += 64) _m_prefetchw(const_cast<uint8_t*>(p + o));
          __atomic_store_n(flags + fs * 16, static_cast<uint32_t>(fin), __ATOMIC_RELEASE);
          ++fin;
          continue;
        }
      }
      const int s = static_cast<int>((next - 1) % a.slots);
      if (posted[s].load(std::memory_order_acquire) != next ||
          (m != 0 && a.lag > 0 && !draining.load(std::memory_order_acquire) &&
           last_posted.load(std::memory_order_acquire) < next + static_cast<uint64_t>(a.lag))) {
        _mm_pause();
        continue;
      }
      uint8_t* dst = hbm + ((next - 1) % (a.slots * 8)) * a.slot;
      uint8_t* slot = ring + s * a.slot;
      if (m == 0) {
        __atomic_store_n(flags + s * 16, static_cast<uint32_t>(next), __ATOMIC_RELEASE);
      } else if (m == 7 || m == 8) {
        uint8_t* vd = vland + ((next - 1) % (a.slots * 8)) * a.slot;
        if (m == 7)
          rep_movsb(vd, slot, a.slot);
        else
          nt_copy(vd, slot, a.slot);
        __atomic_store_n(flags + s * 16, static_cast<uint32_t>(next), __ATOMIC_RELEASE);
      } else {
        if (m == 4) clwb_range(slot, a.slot);
        if (m == 5) flush_range(slot, a.slot);
        if (m == 2 || m == 4 || m == 5 || m == 6)
          check(hipMemcpyAsync(dst, slot, a.slot, hipMemcpyHostToDevice, st[s]), "hipMemcpyAsync");
        else if (m == 3)
          pull_kernel<<<256, 256, 0, st[s]>>>(reinterpret_cast<const uint4*>(ring_d + s * a.slot),
                                              reinterpret_cast<uint4*>(dst), a.slot / 16);
        flag_kernel<<<1, 64, 0, st[s]>>>(
            reinterpret_cast<volatile uint32_t*>((m == 6 ? dflags_d : flags_d) + s * 16), static_cast<uint32_t>(next));
      }
      issued_upto.store(next, std::memory_order_release);
      ++next;
      if (m != 6) fin = next;
    }
  });

  const std::map<std::string, int> dev_code{{"idle", 0},       {"flag", 1},       {"sdma", 2}, {"kernel", 3},
                                            {"sdma_clwb", 4}, {"sdma_flush", 5}, {"sdma_pw", 6},
                                            {"relay", 7},     {"relaynt", 8}};
  const std::map<std::string, int> wr_code{{"memcpy", 0}, {"rep", 1}, {"nt", 2}, {"flush", 3}, {"tcp", 4},
                                           {"tcpv", 5}, {"repv", 6}};
  // fine-grained VRAM for the tcpv / repv writers, if the host can store to it
  uint8_t* vram = nullptr;
  bool vram_ok = false;
  for (const auto& v : a.variants)
    if (v.rfind("tcpv", 0) == 0 || v.rfind("repv", 0) == 0) {
      if (hipExtMallocWithFlags(reinterpret_cast<void**>(&vram), a.slot * a.slots, hipDeviceMallocFinegrained) ==
          hipSuccess)
        vram_ok = host_writable(vram);
      std::printf("{\"vram\": \"finegrained\", \"allocated\": %s, \"host_writable\": %s}\n", vram ? "true" : "false",
                  vram_ok ? "true" : "false");
      std::fflush(stdout);
      break;
    }

  // the loopback connection for the tcp writer: the sender sends `total`
  // bytes per go, from the THP source by vmsplice + splice
  int lfd = socket(AF_INET, SOCK_STREAM, 0), cfd = -1;
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (lfd < 0 || bind(lfd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || listen(lfd, 1) != 0) return 2;
  socklen_t sl_ = sizeof(sa);
  getsockname(lfd, reinterpret_cast<sockaddr*>(&sa), &sl_);
  cfd = socket(AF_INET, SOCK_STREAM, 0);
  if (connect(cfd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0) return 2;
  const int afd = accept(lfd, nullptr, nullptr);
  if (afd < 0) return 2;
  {
    int one = 1;
    setsockopt(afd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  std::atomic<int> send_go{0};
  std::thread sender([&] {
    pin(a.sender);
    int q[2];
    if (pipe2(q, O_CLOEXEC) != 0) return;
    (void)fcntl(q[1], F_SETPIPE_SZ, 1 << 20);
    size_t off = 0;
    for (int done = 0;;) {
      while (send_go.load(std::memory_order_acquire) == done) usleep(100);
      if (send_go.load() < 0) break;
      ++done;
      for (size_t sent = 0; sent < a.total;) {
        if (off >= a.src_bytes) off = 0;
        const size_t k = std::min<size_t>({a.total - sent, a.src_bytes - off, size_t(2) << 20});
        iovec iov{src + off, k};
        const ssize_t v = vmsplice(q[1], &iov, 1, 0);
        if (v <= 0) return;
        for (ssize_t left = v; left > 0;) {
          const ssize_t w = splice(q[0], nullptr, afd, nullptr, static_cast<size_t>(left), SPLICE_F_MOVE | SPLICE_F_MORE);
          if (w <= 0) return;
          left -= w;
        }
        off += static_cast<size_t>(v);
        sent += static_cast<size_t>(v);
      }
    }
    close(q[0]);
    close(q[1]);
  });
  uint64_t seq = 0;
  size_t src_off = 0;
  for (int rep = 0; rep < a.reps; ++rep) {
    for (size_t vi = 0; vi < a.variants.size(); ++vi) {
      const std::string& v = a.variants[(vi + rep) % a.variants.size()];  // rotate the order per rep
      const size_t sl = v.find('/');
      if (sl == std::string::npos || !wr_code.count(v.substr(0, sl)) || !dev_code.count(v.substr(sl + 1))) {
        std::fprintf(stderr, "unknown variant %s\n", v.c_str());
        continue;
      }
      const int wm = wr_code.at(v.substr(0, sl));
      if ((wm == 5 || wm == 6) && !vram_ok) continue;
      const int m = dev_code.at(v.substr(sl + 1));
      if ((m == 7 || m == 8) && !vland_ok) continue;
      mode.store(m, std::memory_order_release);
      std::vector<int> wcpus{a.writer};
      if (a.writer >= 0 && sibling_of(a.writer) >= 0) wcpus.push_back(sibling_of(a.writer));
      const auto irq0 = irqs_on(wcpus);
      int64_t wait_ns = 0, copy_ns = 0;
      double writer_cpu = 0;
      if (wm == 4 || wm == 5) send_go.fetch_add(1, std::memory_order_release);
      draining.store(false, std::memory_order_release);
      std::thread w([&] {
        pin(a.writer);
        const int64_t c0 = thread_cpu_ns();
        const size_t n = a.total / a.slot;
        for (size_t i = 0; i < n; ++i) {
          ++seq;
          const int s = static_cast<int>((seq - 1) % a.slots);
          uint8_t* p = (wm == 5 || wm == 6 ? vram : ring) + s * a.slot;
          // the slot is free once the device finished its previous use
          if (seq > static_cast<uint64_t>(a.slots)) {
            const uint32_t want = static_cast<uint32_t>(seq - a.slots);
            const int64_t t0 = now_ns();
            while (__atomic_load_n(flags + s * 16, __ATOMIC_ACQUIRE) != want) _mm_pause();
            wait_ns += now_ns() - t0;
          }
          const int64_t t1 = now_ns();
          if (src_off + a.slot > a.src_bytes) src_off = 0;
          if (wm == 4 || wm == 5) {
            for (size_t got = 0; got < a.slot;) {
              const ssize_t r = recv(cfd, p + got, a.slot - got, 0);
              if (r <= 0) {
                std::fprintf(stderr, "recv failed\n");
                std::exit(3);
              }
              got += static_cast<size_t>(r);
            }
          } else if (wm == 2)
            nt_copy(p, src + src_off, a.slot);
          else if (wm == 1 || wm == 6)
            rep_movsb(p, src + src_off, a.slot);
          else
            std::memcpy(p, src + src_off, a.slot);
          if (wm == 3) flush_range(p, a.slot);
          copy_ns += now_ns() - t1;
          src_off += a.slot;
          posted[s].store(seq, std::memory_order_release);
          last_posted.store(seq, std::memory_order_release);
        }
        draining.store(true, std::memory_order_release);
        // drain: the last slots' device work
        for (int k = 0; k < a.slots; ++k) {
          const uint64_t q = seq - k;
          const int s = static_cast<int>((q - 1) % a.slots);
          while (__atomic_load_n(flags + s * 16, __ATOMIC_ACQUIRE) != static_cast<uint32_t>(q)) _mm_pause();
        }
        writer_cpu = (thread_cpu_ns() - c0) / 1e9;
      });
      const int64_t t0 = now_ns();
      w.join();
      const double el = (now_ns() - t0) / 1e9;
      const double gib = a.total / double(1ull << 30);
      const auto irq1 = irqs_on(wcpus);
      std::string irq_json;
      uint64_t irq_total = 0;
      for (const auto& kv : irq1) {
        const auto it = irq0.find(kv.first);
        const uint64_t d = kv.second - (it == irq0.end() ? 0 : it->second);
        if (!d) continue;
        irq_total += d;
        irq_json += (irq_json.empty() ? "" : ", ") + std::string("\"") + kv.first + "\": " + std::to_string(d);
      }
      std::printf("{\"rep\": %d, \"variant\": \"%s\", \"writer_irqs\": %llu, \"writer_irqs_by_source\": {%s}}\n", rep,
                  v.c_str(), static_cast<unsigned long long>(irq_total), irq_json.c_str());
      std::printf(
          "{\"rep\": %d, \"variant\": \"%s\", \"slots\": %d, \"slot\": %zu, \"lag\": %d, \"GB/s\": %.2f, "
          "\"copy_GB/s\": %.2f, \"copy_s_per_gib\": %.4f, \"wait_s_per_gib\": %.4f, \"writer_cpu_s_per_gib\": %.4f}\n",
          rep, v.c_str(), a.slots, a.slot, a.lag, a.total / el / 1e9, a.total / (copy_ns / 1e9) / 1e9, copy_ns / 1e9 / gib,
          wait_ns / 1e9 / gib, writer_cpu / gib);
      std::fflush(stdout);
    }
  }
  mode.store(-2);
  sub.join();
  send_go.store(-1);
  shutdown(afd, SHUT_RDWR);
  sender.join();
  close(afd);
  close(cfd);
  close(lfd);
  for (auto& s : st) (void)hipStreamDestroy(s);
  (void)hipFree(hbm);
  (void)hipHostFree(flags);
  (void)hipHostFree(dflags);
  if (vram) (void)hipFree(vram);
  if (vland) (void)hipFree(vland);
  (void)hipHostFree(ring);
  munmap(src, a.src_bytes);
  return 0;
}
