// GPU sink: pinned ring -> hipMemcpyAsync -> HBM + CRC32C kernels.  See engine.h.
#include "gpu/engine.h"

#include <algorithm>
#include <cctype>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <numeric>
#include <thread>
#include <stdexcept>

#include <sched.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <time.h>
#include <unistd.h>

#include "core/affinity.h"
#include "core/crc32c.h"
#include "core/util.h"
#include "gpu/markers.h"

namespace gcsb {

namespace {
bool debug_ring() {
  static bool d = [] {
    const char* e = std::getenv("GCSB_DEBUG_RING");
    return e && *e == '1';
  }();
  return d;
}

// Per-device resources reused across calls: a stream for one-off CRC jobs,
// host-mapped result slots and a tile scratch buffer.  Creating these per
// call (streams, hipHostMalloc, hipMalloc) cost milliseconds per upload.
struct DeviceCtx {
  std::mutex mu;  // one gpu_crc32c job at a time per device
  hipStream_t st = nullptr;
  CrcSegResult* res = nullptr;
  CrcSegResult* d_res = nullptr;
  uint32_t* d_tiles = nullptr;
  size_t tiles_cap = 0;
};

DeviceCtx& device_ctx(int dev) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<DeviceCtx>> ctx;
  std::lock_guard<std::mutex> lk(mu);
  auto& c = ctx[dev];
  if (!c) {
    auto n = std::make_unique<DeviceCtx>();
    hip_check(hipStreamCreateWithFlags(&n->st, hipStreamNonBlocking), "hipStreamCreate");
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&n->res), sizeof(CrcSegResult) * kMaxSeg,
                            hipHostMallocMapped | hipHostMallocCoherent),
              "hipHostMalloc(results)");
    hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&n->d_res), n->res, 0), "hipHostGetDevicePointer");
    c = std::move(n);
  }
  return *c;
}

// Page-locked staging buffers recycled by size (upload rings, per-call
// sinks): hipHostMalloc of tens of MiB is far slower than the D2H it feeds.
//
// Page-locked memory is 2 MiB-aligned anonymous memory with MADV_HUGEPAGE,
// first-touched by the calling (GPU-local, pinned) thread, then
// hipHostRegister'ed.  The receiving core's copy_to_user writes every object
// byte into these pages, so 512x fewer TLB misses per slot than
// hipHostMalloc's 4 KiB pages is on the one-stream critical path; the SDMA
// engine reads them through the same IOMMU mappings either way.
// hipHostMalloc(NumaUser) is the fallback when registration fails.

// NUMA node of a HIP device's PCIe root (sysfs), -1 if unknown; cached.
int device_numa_node(int dev) {
  static std::mutex mu;
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int node = -1;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) == hipSuccess) {
    for (char* c = bus; *c; ++c) *c = static_cast<char>(std::tolower(static_cast<unsigned char>(*c)));
    if (FILE* f = std::fopen((std::string("/sys/bus/pci/devices/") + bus + "/numa_node").c_str(), "r")) {
      if (std::fscanf(f, "%d", &node) != 1) node = -1;
      std::fclose(f);
    }
  } else {
    (void)hipGetLastError();
  }
  cache[dev] = node;
  return node;
}

class PinnedPool {
 public:
  // n bytes of page-locked memory whose pages sit on NUMA node `node` (the
  // GPU's, which its SDMA engines read / write and its rank's pinned threads
  // run on), -1 = the calling thread's node.  Recycled by (node, size).
  // wc: a read sink's ring, which the CPU only writes (the receive copy) and
  // the copy engine reads, in write-combined memory
  // (hipHostMallocWriteCombined, not pooled): the copy's stores skip the CPU
  // caches, so there is no read-for-ownership and nothing to write back
  // before the DMA (GpuSinkConfig::ring_wc).  Never for upload staging,
  // which the CPU reads.
  static void* get(size_t n, int node, bool wc = false) {
    if (wc) {
      void* p = nullptr;
      hip_check(hipHostMalloc(&p, n, hipHostMallocWriteCombined | hipHostMallocNumaUser), "hipHostMalloc(wc ring)");
      std::lock_guard<std::mutex> lk(mu());
      wc_set()[p] = n;
      return p;
    }
    if (node < 0) node = current_numa_node();
    {
      std::lock_guard<std::mutex> lk(mu());
      auto it = free_list().find({node, n});
      if (it != free_list().end()) {
        void* p = it->second;
        free_list().erase(it);
        held() -= n;
        return p;
      }
    }
    {
      const size_t huge = size_t(2) << 20;
      const size_t len = (n + huge - 1) / huge * huge;
      // a fresh mapping, never touched: malloc'd memory (even 2 MiB-aligned)
      // can reuse pages another thread already faulted in on the other
      // socket, which no memory policy moves (bench numa.ring_slot_nodes
      // showed slot 0 there in 1 of 3 runs)
      void* raw = ::mmap(nullptr, len + huge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (raw != MAP_FAILED) {
        const uintptr_t a = (reinterpret_cast<uintptr_t>(raw) + huge - 1) & ~(huge - 1);
        const size_t head = a - reinterpret_cast<uintptr_t>(raw);
        if (head) ::munmap(raw, head);
        if (huge - head) ::munmap(reinterpret_cast<void*>(a + len), huge - head);
        void* p = reinterpret_cast<void*>(a);
        (void)madvise(p, len, MADV_HUGEPAGE);
        (void)bind_range_to_node(p, len, node);  // strictly, whichever thread faults it in
        std::memset(p, 0, len);  // fault in now
        if (hipHostRegister(p, len, hipHostRegisterDefault) == hipSuccess) {
          std::lock_guard<std::mutex> lk(mu());
          registered()[p] = {len, node};
          return p;
        }
        (void)hipGetLastError();
        ::munmap(p, len);
      }
    }
    void* p = nullptr;
    hip_check(hipHostMalloc(&p, n, hipHostMallocNumaUser), "hipHostMalloc(staging)");
    {
      std::lock_guard<std::mutex> lk(mu());
      malloced()[p] = node;
    }
    return p;
  }
  static void put(void* p, size_t n) {
    if (!p) return;
    size_t reg_len = 0;
    {
      std::lock_guard<std::mutex> lk(mu());
      if (wc_set().erase(p)) {
        (void)hipHostFree(p);
        return;
      }
      auto it = registered().find(p);
      const int node = it != registered().end() ? it->second.second : malloced()[p];
      if (held() + n <= kMaxHeld) {
        free_list().emplace(std::make_pair(node, n), p);
        held() += n;
        return;
      }
      if (it != registered().end()) {
        reg_len = it->second.first;
        registered().erase(it);
      }
      malloced().erase(p);
    }
    if (reg_len) {
      (void)hipHostUnregister(p);
      ::munmap(p, reg_len);
      return;
    }
    (void)hipHostFree(p);
  }

 private:
  static constexpr size_t kMaxHeld = size_t(1) << 30;
  static std::map<void*, std::pair<size_t, int>>& registered() {  // THP ring: length, node
    static std::map<void*, std::pair<size_t, int>> r;
    return r;
  }
  static std::map<void*, int>& malloced() {  // hipHostMalloc fallback: node asked for
    static std::map<void*, int> m;
    return m;
  }
  static std::mutex& mu() {
    static std::mutex m;
    return m;
  }
  static std::map<void*, size_t>& wc_set() {  // write-combined sink rings (not pooled)
    static std::map<void*, size_t> w;
    return w;
  }
  static std::multimap<std::pair<int, size_t>, void*>& free_list() {
    static std::multimap<std::pair<int, size_t>, void*> f;
    return f;
  }
  static size_t& held() {
    static size_t h = 0;
    return h;
  }
};
}  // namespace

// Upload sources (a GpuByteSource per upload, 32 staging slots for a 64 MiB
// object) recycle their completion events instead of creating and
// destroying them per upload.  Per device, flags hipEventDisableTiming.
class EventPool {
 public:
  static hipEvent_t get(int dev) {
    {
      std::lock_guard<std::mutex> lk(mu());
      auto& v = free()[dev];
      if (!v.empty()) {
        hipEvent_t e = v.back();
        v.pop_back();
        return e;
      }
    }
    hipEvent_t e = nullptr;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return e;
  }
  static void put(int dev, hipEvent_t e) {
    if (!e) return;
    std::lock_guard<std::mutex> lk(mu());
    auto& v = free()[dev];
    if (v.size() < 1024) {
      v.push_back(e);
      return;
    }
    (void)hipEventDestroy(e);
  }

 private:
  static std::mutex& mu() {
    static std::mutex m;
    return m;
  }
  static std::map<int, std::vector<hipEvent_t>>& free() {
    static auto* f = new std::map<int, std::vector<hipEvent_t>>();  // process lifetime
    return *f;
  }
};

int gpu_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

namespace {
// hipSetDevice only when this thread's current device differs.
void ensure_device(int dev) {
  thread_local int cur = -1;
  if (cur != dev) {
    hip_check(hipSetDevice(dev), "hipSetDevice");
    cur = dev;
  }
}

std::mutex g_submit_mu;
std::vector<int> g_submit_cpus;
bool g_submit_cpus_set = false;

std::vector<int> submitter_cpus() {
  std::lock_guard<std::mutex> lk(g_submit_mu);
  if (!g_submit_cpus_set) {
    if (const char* e = std::getenv("GCSB_SUBMIT_CPUS")) g_submit_cpus = parse_cpulist(e);
    g_submit_cpus_set = true;
  }
  return g_submit_cpus;
}

// One thread per device that issues every queued ring-slot hand-off, so HIP
// API calls are made by one thread instead of contending from many transport
// threads.  Jobs run in FIFO order; each job is a few async HIP calls.
std::atomic<int> g_submit_spin_us{0};

class DeviceSubmitter {
 public:
  static DeviceSubmitter& get(int dev) {
    static std::mutex mu;
    static std::map<int, DeviceSubmitter*> all;  // process lifetime (never joined at exit)
    std::lock_guard<std::mutex> lk(mu);
    auto& p = all[dev];
    if (!p) p = new DeviceSubmitter(dev);
    return *p;
  }
  // The posting (receiving) thread wakes the submitter only when it sleeps:
  // a futex wake costs the receiving thread microseconds per slot.
  void post(std::function<void()> f) {
    bool wake;
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(f));
      pending_.store(true, std::memory_order_release);
      wake = sleeping_;
    }
    if (wake) cv_.notify_one();
  }

 private:
  explicit DeviceSubmitter(int dev) : dev_(dev) { std::thread([this] { loop(); }).detach(); }
  void loop() {
    name_current_thread("gcsb-submit");
    // off the receiving core: inherited from the first posting thread (a
    // pinned transport thread) it would share that core's SMT pair
    const std::vector<int> cpus = submitter_cpus();
    if (cpus.empty()) {
      // not configured: the process's (main thread's) CPU set, not the first
      // poster's -- a receive thread pinned to one CPU would otherwise hand
      // the submitter its own CPU
      cpu_set_t m;
      CPU_ZERO(&m);
      if (sched_getaffinity(getpid(), sizeof m, &m) == 0) sched_setaffinity(0, sizeof m, &m);
    } else {
      pin_current_thread(cpus);
    }
    ensure_device(dev_);
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      const int spin_us = g_submit_spin_us.load(std::memory_order_relaxed);
      if (q_.empty() && spin_us > 0) {
        // poll for the next hand-off before sleeping: a post to a polling
        // submitter costs the receiving thread no futex wake
        lk.unlock();
        const int64_t until = now_ns() + spin_us * 1000LL;
        while (!pending_.load(std::memory_order_acquire) && now_ns() < until) __builtin_ia32_pause();
        lk.lock();
      }
      if (q_.empty()) {
        sleeping_ = true;
        cv_.wait(lk, [&] { return !q_.empty(); });
        sleeping_ = false;
      }
      auto f = std::move(q_.front());
      q_.pop_front();
      pending_.store(!q_.empty(), std::memory_order_release);
      lk.unlock();
      f();
      lk.lock();
    }
  }
  int dev_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::atomic<bool> pending_{false};
  bool sleeping_ = false;  // guarded by mu_
};
}  // namespace

void set_submitter_spin_us(int us) { g_submit_spin_us.store(std::max(0, us), std::memory_order_relaxed); }

void set_submitter_cpus(const std::vector<int>& cpus) {
  std::lock_guard<std::mutex> lk(g_submit_mu);
  g_submit_cpus = cpus;
  g_submit_cpus_set = true;
}

namespace {
std::mutex g_slow_mu;
SlowHipCalls g_slow;
constexpr int64_t kSlowCallNs = 1000000;

// Records one hand-off HIP call that ran [t0, t1) on the calling thread.
void note_hip_call(const char* what, int stream_idx, int64_t t0, int64_t t1) {
  const int64_t d = t1 - t0;
  std::lock_guard<std::mutex> lk(g_slow_mu);
  ++g_slow.calls;
  if (d < kSlowCallNs) return;
  ++g_slow.slow;
  g_slow.slow_ms_total += d / 1e6;
  if (d / 1e6 > g_slow.max_ms) {
    g_slow.max_ms = d / 1e6;
    g_slow.max_call = std::string(what) + " stream " + std::to_string(stream_idx);
  }
}
}  // namespace

SlowHipCalls slow_hip_calls() {
  std::lock_guard<std::mutex> lk(g_slow_mu);
  return g_slow;
}

void reset_slow_hip_calls() {
  std::lock_guard<std::mutex> lk(g_slow_mu);
  g_slow = SlowHipCalls();
}

// Per-device stream pool shared by every sink / upload source (engine.h).
class DeviceStreamPool {
 public:
  static DeviceStreamPool& get(int dev) {
    static std::mutex mu;
    static std::map<int, DeviceStreamPool*> all;  // process lifetime
    std::lock_guard<std::mutex> lk(mu);
    auto& p = all[dev];
    if (!p) p = new DeviceStreamPool(dev);
    return *p;
  }
  hipStream_t at(unsigned i) const { return st_[i % st_.size()]; }
  unsigned next_base() { return rr_.fetch_add(1); }
  size_t size() const { return st_.size(); }
  int index_of(hipStream_t s) const {
    for (size_t i = 0; i < st_.size(); ++i)
      if (st_[i] == s) return static_cast<int>(i);
    return -1;
  }
  // GCSB_STREAMS=0: no pool, every sink / source owns one private stream
  // (A/B switch against the shared pool).
  bool private_streams() const { return st_.empty(); }

 private:
  explicit DeviceStreamPool(int dev) {
    // 8: sliced reads (16 sinks) p99 6.0-6.2 ms vs 6.7-13.3 with 4 and
    // 10-16 with a private stream per sink; one stream per read: equal within
    // run-to-run spread (profiles/r2_streams_ab)
    int n = 8;
    if (const char* e = std::getenv("GCSB_STREAMS")) n = std::max(0, std::min(32, std::atoi(e)));
    ensure_device(dev);
    // every SDMA engine up before the first read / upload can land on a cold
    // one (gpu/copy_engines.hip)
    (void)warm_copy_engines(dev);
    st_.resize(static_cast<size_t>(n));
    for (auto& st : st_) hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate(pool)");
  }
  std::vector<hipStream_t> st_;
  std::atomic<unsigned> rr_{0};
};

void warm_device_streams(int device) {
  ensure_device(device);
  DeviceStreamPool& pool = DeviceStreamPool::get(device);
  static std::mutex mu;
  static std::map<int, std::pair<uint8_t*, uint8_t*>> bufs;  // per device: pinned host, HBM scratch
  std::lock_guard<std::mutex> lk(mu);
  auto& b = bufs[device];
  if (!b.first) {
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&b.first), 8192, hipHostMallocDefault), "hipHostMalloc(warm)");
    hip_check(hipMalloc(reinterpret_cast<void**>(&b.second), 8192), "hipMalloc(warm)");
  }
  for (size_t i = 0; i < pool.size(); ++i) {
    hipStream_t st = pool.at(static_cast<unsigned>(i));
    const int64_t t0 = now_ns();
    hip_check(hipMemcpyAsync(b.second, b.first, 4096, hipMemcpyHostToDevice, st), "hipMemcpyAsync(warm H2D)");
    const int64_t t1 = now_ns();
    note_hip_call("warm hipMemcpyAsync(H2D)", static_cast<int>(i), t0, t1);
    hip_check(hipMemcpyAsync(b.first + 4096, b.second, 4096, hipMemcpyDeviceToHost, st), "hipMemcpyAsync(warm D2H)");
    note_hip_call("warm hipMemcpyAsync(D2H)", static_cast<int>(i), t1, now_ns());
  }
  for (size_t i = 0; i < pool.size(); ++i)
    hip_check(hipStreamSynchronize(pool.at(static_cast<unsigned>(i))), "hipStreamSynchronize(warm)");
}

CopyCeiling copy_ceiling(int device, bool h2d, size_t total, size_t chunk, int slots, int streams, int iters) {
  ensure_device(device);
  if (chunk == 0 || total == 0 || slots < 1 || iters < 1) throw std::invalid_argument("copy_ceiling: bad geometry");
  DeviceStreamPool& pool = DeviceStreamPool::get(device);
  const unsigned nst = static_cast<unsigned>(std::max(1, std::min(streams, std::max(1, static_cast<int>(pool.size())))));
  std::vector<uint8_t*> host(slots);
  std::vector<hipEvent_t> ev(slots, nullptr);
  std::vector<bool> busy(slots, false);
  uint8_t* dev = nullptr;
  hip_check(hipMalloc(reinterpret_cast<void**>(&dev), total), "hipMalloc(copy ceiling)");
  for (int i = 0; i < slots; ++i) {
    host[i] = static_cast<uint8_t*>(PinnedPool::get(chunk, device_numa_node(device)));
    hip_check(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming), "hipEventCreate");
  }
  hipStream_t priv = nullptr;
  if (pool.private_streams()) hip_check(hipStreamCreateWithFlags(&priv, hipStreamNonBlocking), "hipStreamCreate");
  std::vector<double> pass_ms;
  double timed_s = 0;
  for (int it = 0; it <= iters; ++it) {
    const int64_t t0 = now_ns();
    size_t k = 0;
    for (size_t off = 0; off < total; off += chunk, ++k) {
      const int i = static_cast<int>(k % static_cast<size_t>(slots));
      if (busy[i]) hip_check(hipEventSynchronize(ev[i]), "hipEventSynchronize");
      hipStream_t st = priv ? priv : pool.at(static_cast<unsigned>(k) % nst);
      const size_t n = std::min(chunk, total - off);
      if (h2d)
        hip_check(hipMemcpyAsync(dev + off, host[i], n, hipMemcpyHostToDevice, st), "hipMemcpyAsync(H2D)");
      else
        hip_check(hipMemcpyAsync(host[i], dev + off, n, hipMemcpyDeviceToHost, st), "hipMemcpyAsync(D2H)");
      hip_check(hipEventRecord(ev[i], st), "hipEventRecord");
      busy[i] = true;
    }
    for (int i = 0; i < slots; ++i)
      if (busy[i]) {
        hip_check(hipEventSynchronize(ev[i]), "hipEventSynchronize");
        busy[i] = false;
      }
    const double s = (now_ns() - t0) / 1e9;
    if (it > 0) {  // pass 0 is the untimed warm-up
      timed_s += s;
      pass_ms.push_back(s * 1e3);
    }
  }
  for (int i = 0; i < slots; ++i) {
    PinnedPool::put(host[i], chunk);
    (void)hipEventDestroy(ev[i]);
  }
  (void)hipFree(dev);
  if (priv) (void)hipStreamDestroy(priv);
  std::sort(pass_ms.begin(), pass_ms.end());
  CopyCeiling r;
  r.gbps = static_cast<double>(total) * iters / timed_s / 1e9;
  r.pass_ms_p50 = pass_ms[pass_ms.size() / 2];
  return r;
}

void GpuSink::set_device() const { ensure_device(cfg_.device); }

GpuSink::GpuSink(const GpuSinkConfig& cfg) : cfg_(cfg) {
  if (cfg_.stage != GpuSinkConfig::Stage::kH2D) cfg_.verify = false;
  if (cfg_.slots < 2) cfg_.slots = 2;
  cfg_.slot_bytes = (cfg_.slot_bytes + 4095) / 4096 * 4096;
  if (cfg_.slot_bytes < 65536) cfg_.slot_bytes = 65536;
  set_device();
  if (cfg_.conn_ring) {
    // the connection's ring is the receive destination: no private ring
    if (cfg_.landing != Landing::kObject || !cfg_.verify || cfg_.stage != GpuSinkConfig::Stage::kH2D)
      throw std::invalid_argument("GpuSink: conn_ring needs object landing with CRC verification");
    if (cfg_.conn_ring->device() != cfg_.device) throw std::invalid_argument("GpuSink: conn_ring on another device");
    return;
  }
  DeviceStreamPool& pool = DeviceStreamPool::get(cfg_.device);
  // Slot i of a sink uses pool stream i (slot i's CRC overlaps slot i+1's
  // copy; the sliced block's 16 sinks spread over all 8).  Alternating a
  // sink's slots over 2 streams instead cost the sliced block 7-9% and did
  // not hold the first-read tail lower (profiles/r2_streams_sync).
  const unsigned nst = static_cast<unsigned>(cfg_.slots);
  const unsigned base = pool.next_base() * nst;
  if (pool.private_streams())
    hip_check(hipStreamCreateWithFlags(&own_stream_, hipStreamNonBlocking), "hipStreamCreate");
  d_tables_ = device_crc_tables(cfg_.device);
  tiles_cap_ = cfg_.slot_bytes / kCrcMinTile + 2 * kMaxSeg + 8;
  d_tiles_ = crc_scratch_alloc(crc_scratch_words(tiles_cap_) * cfg_.slots);
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&res_host_), sizeof(CrcSegResult) * kMaxSeg * cfg_.slots,
                          hipHostMallocMapped | hipHostMallocCoherent),
            "hipHostMalloc(results)");
  std::memset(res_host_, 0, sizeof(CrcSegResult) * kMaxSeg * cfg_.slots);
  slots_.resize(cfg_.slots);
  for (int i = 0; i < cfg_.slots; ++i) {
    Slot& s = slots_[i];
    // on the GPU's NUMA node (the rank's pinned receive thread runs there too)
    if (!cfg_.ring_wc && i == 0)
      ring_base_ = static_cast<uint8_t*>(PinnedPool::get(cfg_.slot_bytes * cfg_.slots, device_numa_node(cfg_.device)));
    s.host = ring_base_ ? ring_base_ + cfg_.slot_bytes * static_cast<size_t>(i)
                        : static_cast<uint8_t*>(PinnedPool::get(cfg_.slot_bytes, device_numa_node(cfg_.device), true));
    if (cfg_.landing == Landing::kRing)
      hip_check(hipMalloc(reinterpret_cast<void**>(&s.dev_ring), cfg_.slot_bytes), "hipMalloc(ring slot)");
    const unsigned evf = hipEventDisableTiming | (cfg_.blocking_sync ? hipEventBlockingSync : 0u);
    hip_check(hipEventCreateWithFlags(&s.ev, evf), "hipEventCreate");
    s.st = own_stream_ ? own_stream_ : pool.at(base + static_cast<unsigned>(i) % nst);
    s.st_idx = own_stream_ ? -1 : pool.index_of(s.st);
    s.tiles = d_tiles_ + crc_scratch_words(tiles_cap_) * static_cast<size_t>(i);
    s.res = res_host_ + static_cast<size_t>(i) * kMaxSeg;
    hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.d_res), s.res, 0), "hipHostGetDevicePointer");
  }
}

GpuSink::~GpuSink() {
  try {
    if (cfg_.conn_ring) ring_wait_all();    // no segment of this sink may outlive it
    for (Slot& sl : slots_) wait_slot(sl);  // no queued hand-off may outlive the sink
    set_device();
  } catch (...) {
  }
  if (ring_base_) PinnedPool::put(ring_base_, cfg_.slot_bytes * cfg_.slots);
  for (Slot& s : slots_) {
    if (!ring_base_) PinnedPool::put(s.host, cfg_.slot_bytes);
    if (s.dev_ring) (void)hipFree(s.dev_ring);
    if (s.ev) (void)hipEventDestroy(s.ev);
  }
  if (res_host_) (void)hipHostFree(res_host_);
  if (d_tiles_) (void)hipFree(d_tiles_);
  if (own_obj_) (void)hipFree(own_obj_);
  if (own_stream_) (void)hipStreamDestroy(own_stream_);
}

void GpuSink::set_external_destination(void* dptr, size_t cap) {
  set_device();
  if (cfg_.conn_ring) ring_wait_all();    // this sink's segments in the connection's ring
  for (Slot& sl : slots_) wait_slot(sl);  // this sink's queued work (its slot events), not the shared streams
  if (own_obj_) {
    (void)hipFree(own_obj_);
    own_obj_ = nullptr;
  }
  obj_dst_ = static_cast<uint8_t*>(dptr);
  obj_cap_ = cap;
  external_dst_ = dptr != nullptr;
}

void GpuSink::ensure_object_capacity(int64_t size) {
  if (cfg_.landing != Landing::kObject || size < 0) return;
  uint64_t need = static_cast<uint64_t>(size) - static_cast<uint64_t>(info_.start_offset);
  if (need <= obj_cap_) return;
  grow_object_buffer(need);
}

// Re-allocates the sink-owned HBM landing buffer, preserving the bytes that
// already landed (gRPC learns the object size only from the first message's
// metadata, after its content).  Happens once per sink: later reads reuse it.
void GpuSink::grow_object_buffer(uint64_t need) {
  if (external_dst_)
    throw StorageError("object larger than the external HBM destination (" + std::to_string(obj_cap_) + " B)", false);
  set_device();
  uint64_t landed = delivered_;
  if (cfg_.conn_ring) {
    ring_wait_all();  // every landed byte's copy done before the old buffer goes
  } else {
    for (int k = 0; k < cfg_.slots; ++k) wait_slot(slots_[(next_ + k) % cfg_.slots]);
    landed = cur_ >= 0 ? slots_[cur_].obj_off : delivered_;
  }
  size_t cap = (need + (2u << 20) - 1) / (2u << 20) * (2u << 20);
  uint8_t* nb = nullptr;
  hip_check(hipMalloc(reinterpret_cast<void**>(&nb), cap), "hipMalloc(object landing)");
  if (own_obj_) {
    if (landed) hip_check(hipMemcpy(nb, own_obj_, landed, hipMemcpyDeviceToDevice), "hipMemcpy(D2D grow)");
    hip_check(hipFree(own_obj_), "hipFree");
  }
  own_obj_ = nb;
  obj_dst_ = own_obj_;
  obj_cap_ = cap;
}

void GpuSink::begin(const ObjectInfo& info) {
  abort();  // drain anything a previous (failed) read left behind
  if (cfg_.conn_ring) {
    std::lock_guard<std::mutex> lk(cfg_.conn_ring->mu_);
    ring_res_.clear();
    ring_done_ = 0;
    ring_open_slot_ = -1;
    chunks_.clear();
  }
  info_ = info;
  delivered_ = 0;
  in_chunk_ = false;
  chunk_start_pending_ = false;
  chunk_broken_ = false;
  chunk_raw_ = 0;
  chunk_len_ = 0;
  obj_raw_ = 0;
  obj_len_ = 0;
  mismatch_ = false;
  any_checked_ = false;
  detail_.clear();
  ensure_object_capacity(info.size);
}

void GpuSink::update_info(const ObjectInfo& info) {
  if (info.has_crc32c) {
    info_.has_crc32c = true;
    info_.crc32c = info.crc32c;
  }
  if (!info.md5.empty()) info_.md5 = info.md5;
  if (info.generation) info_.generation = info.generation;
  if (info.size >= 0 && info_.size < 0) {
    info_.size = info.size;
    ensure_object_capacity(info.size);
  }
}

// The slot's CRC kernel stored every segment's status in host-mapped memory
// (kCrcStatusPending otherwise): the kernel ran after the slot's H2D copy on
// its stream, so the pinned slot is free to refill and its results are final
// -- known without a HIP call (hipEventQuery) on the receiving thread.
bool GpuSink::done_by_flags(const Slot& s) const {
  if (!cfg_.verify || s.segs.empty() || cfg_.stage != GpuSinkConfig::Stage::kH2D) return false;
  for (size_t i = 0; i < s.segs.size(); ++i)
    if (__atomic_load_n(&s.res[i].status, __ATOMIC_ACQUIRE) == kCrcStatusPending) return false;
  return true;
}

GpuSink::Slot& GpuSink::take_slot() {
  const int64_t h0 = now_ns();
  Slot& s = slots_[next_];
  if (s.inflight && done_by_flags(s)) {
    s.inflight = false;
    ++stats_.flag_reuses;
    harvest(s);
  }
  if (s.inflight) {
    ++stats_.slot_waits;
    int64_t t0 = now_ns();
    wait_slot(s);
    stats_.slot_wait_s += (now_ns() - t0) / 1e9;
  }
  s.used = 0;
  s.segs.clear();
  s.obj_off = delivered_;
  cur_ = next_;
  next_ = (next_ + 1) % cfg_.slots;
  stats_.handoff_s += (now_ns() - h0) / 1e9;
  return s;
}

void GpuSink::open_seg(Slot& s) {
  if (!s.segs.empty() && !s.segs.back().closed) return;
  SegInfo g;
  g.slot_off = s.used;
  g.obj_off = delivered_;
  g.chunk_start = chunk_start_pending_;
  g.broken_chunk = chunk_broken_;
  chunk_start_pending_ = false;
  s.segs.push_back(g);
}

Window GpuSink::acquire(size_t want) {
  (void)want;
  if (cfg_.conn_ring) return ring_acquire();
  if (cur_ < 0) take_slot();
  {
    Slot& s = slots_[cur_];
    bool segs_full = s.segs.size() >= static_cast<size_t>(kMaxSeg) && (s.segs.empty() || s.segs.back().closed);
    if (s.used == cfg_.slot_bytes || segs_full) {
      submit_current();
      take_slot();
    }
  }
  Slot& s = slots_[cur_];
  open_seg(s);
  size_t cap = cfg_.slot_bytes - s.used;
  if (cfg_.landing == Landing::kObject) {
    if (delivered_ >= obj_cap_) {
      // size unknown so far (or larger than announced): grow, keeping landed bytes
      grow_object_buffer(std::max<uint64_t>(2 * obj_cap_, delivered_ + cfg_.slot_bytes));
    }
    if (obj_cap_ - delivered_ < cap) cap = obj_cap_ - delivered_;
  }
  // The ring is one contiguous region: when the next slot is free, the
  // window runs on into it, so one recv() is not cut at a slot boundary
  // (648 KiB per recv into 1 MiB slots against 954 KiB into the discard
  // sink's 2 MiB blocks, profiles/r4_final1); commit() splits the bytes.
  spill_ = false;
  if (ring_base_ && cfg_.ring_span && cur_ + 1 < cfg_.slots && next_ == cur_ + 1 && cap == cfg_.slot_bytes - s.used &&
      s.segs.size() < static_cast<size_t>(kMaxSeg)) {
    Slot& n = slots_[next_];
    if (n.inflight && done_by_flags(n)) {
      n.inflight = false;
      ++stats_.flag_reuses;
      harvest(n);
    }
    if (!n.inflight) {
      size_t more = cfg_.slot_bytes;
      if (cfg_.landing == Landing::kObject && obj_cap_ - delivered_ - cap < more) more = obj_cap_ - delivered_ - cap;
      if (more > 0) {
        cap += more;
        spill_ = true;
      }
    }
  }
  // keep a segment below 4 GiB (32-bit length in the kernel batch)
  return Window{s.host + s.used, cap};
}

void GpuSink::commit(size_t n) {
  if (cfg_.conn_ring) return ring_commit(n);
  if (spill_) {
    spill_ = false;
    const size_t room = cfg_.slot_bytes - slots_[cur_].used;
    if (n > room) {
      // the recv ran on into the next slot: this slot is full, the rest of
      // the bytes already sit at the start of the next one
      commit(room);
      submit_current();
      take_slot();
      open_seg(slots_[cur_]);
      commit(n - room);
      return;
    }
  }
  Slot& s = slots_[cur_];
  if (debug_ring() && (s.segs.empty() || s.segs.back().closed || s.used + n > cfg_.slot_bytes))
    throw std::logic_error("GpuSink::commit outside an acquired window");
  s.used += n;
  s.segs.back().len += static_cast<uint32_t>(n);
  delivered_ += n;
}

void GpuSink::chunk_begin(size_t len) {
  if (cfg_.conn_ring) {
    // a segment never spans two chunks: the host fold checks each chunk
    std::lock_guard<std::mutex> lk(cfg_.conn_ring->mu_);
    ring_open_slot_ = -1;
    if (!chunks_.empty() && !chunks_.back().closed) {  // the last chunk never ended: unverifiable
      chunks_.back().closed = true;
      chunks_.back().broken = true;
      chunks_.back().end = delivered_;
    }
    ChunkMark m;
    m.start = m.end = delivered_;
    chunks_.push_back(m);
    return;
  }
  if (cur_ >= 0) {
    Slot& s = slots_[cur_];
    if (!s.segs.empty()) s.segs.back().closed = true;
    // keep a chunk inside one slot when it fits, so its CRC is checked in
    // the K2 epilogue on the GPU instead of being folded on the host
    if (s.used > 0 && cfg_.slot_bytes - s.used < len && len <= cfg_.slot_bytes) submit_current();
  }
  in_chunk_ = true;
  chunk_start_pending_ = true;
  chunk_broken_ = false;
}

void GpuSink::chunk_end(bool has_crc, uint32_t crc) {
  if (cfg_.conn_ring) {
    std::lock_guard<std::mutex> lk(cfg_.conn_ring->mu_);
    ring_open_slot_ = -1;
    if (chunks_.empty() || chunks_.back().closed) return;
    ChunkMark& m = chunks_.back();
    m.end = delivered_;
    m.closed = true;
    m.has_crc = has_crc;
    m.crc = crc;
    return;
  }
  if (!in_chunk_) return;
  in_chunk_ = false;
  if (chunk_start_pending_) {
    // zero-length chunk: nothing landed
    chunk_start_pending_ = false;
    if (has_crc && cfg_.verify) {
      any_checked_ = true;
      if (crc != 0) {
        mismatch_ = true;
        detail_ = "empty chunk with non-zero crc32c";
      }
    }
    return;
  }
  if (cur_ < 0 || slots_[cur_].segs.empty() || slots_[cur_].segs.back().closed) return;
  SegInfo& g = slots_[cur_].segs.back();
  g.closed = true;
  g.chunk_end = true;
  g.has_expected = has_crc;
  g.expected = crc;
  g.broken_chunk = chunk_broken_;
}

void GpuSink::resume_at(int64_t offset) {
  (void)offset;
  if (cfg_.conn_ring) {
    std::lock_guard<std::mutex> lk(cfg_.conn_ring->mu_);
    ring_open_slot_ = -1;
    if (!chunks_.empty() && !chunks_.back().closed) {
      chunks_.back().closed = true;
      chunks_.back().broken = true;
      chunks_.back().end = delivered_;
    }
    return;
  }
  chunk_broken_ = true;
  if (cur_ >= 0 && !slots_[cur_].segs.empty() && !slots_[cur_].segs.back().closed) {
    slots_[cur_].segs.back().closed = true;
    slots_[cur_].segs.back().broken_chunk = true;
  }
  in_chunk_ = false;
  chunk_start_pending_ = false;
}

void GpuSink::submit_current() {
  if (cur_ < 0) return;
  RoctxRange rg("gcsb.slot_submit");
  struct Timed {
    double* acc;
    int64_t t0 = now_ns();
    ~Timed() { *acc += (now_ns() - t0) / 1e9; }
  } timed{&stats_.handoff_s};
  Slot& s = slots_[cur_];
  cur_ = -1;
  if (s.used == 0) {
    // nothing landed: hand the slot back (it is the one next_ points behind)
    next_ = static_cast<int>((next_ + cfg_.slots - 1) % cfg_.slots);
    return;
  }
  if (!s.segs.empty()) s.segs.back().closed = true;
  uint8_t* dst = cfg_.landing == Landing::kObject ? obj_dst_ + s.obj_off : s.dev_ring;
  CrcBatch b;
  const bool crc = cfg_.verify && !s.segs.empty();
  if (crc) {
    std::memset(&b, 0, sizeof(b));
    b.nseg = static_cast<uint32_t>(s.segs.size());
    for (size_t i = 0; i < s.segs.size(); ++i) {
      const SegInfo& g = s.segs[i];
      CrcSeg& c = b.seg[i];
      c.addr = dst + g.slot_off;
      c.len = g.len;
      c.expected = g.expected;
      c.flags = (g.chunk_start && g.chunk_end && g.has_expected && !g.broken_chunk) ? 1u : 0u;
    }
    finalize_crc_batch(&b);
    if (b.total_tiles > tiles_cap_) throw std::logic_error("CRC tile scratch too small");
    stats_.segments += s.segs.size();
    for (size_t i = 0; i < s.segs.size(); ++i) __atomic_store_n(&s.res[i].status, kCrcStatusPending, __ATOMIC_RELAXED);
  }
  s.inflight = true;
  ++stats_.slots_submitted;
  enqueue_slot(s, dst, crc ? &b : nullptr);
}

// The slot's H2D copy, CRC launches and completion event.  Runs on the
// device submitter thread (async_submit) or inline.
void GpuSink::enqueue_slot(Slot& s, uint8_t* dst, const CrcBatch* batch) {
  auto issue = [this, &s, dst](const CrcBatch* b) {
    if (cfg_.stage == GpuSinkConfig::Stage::kHostRead) {
      host_read_sink_ = crc32c_extend(host_read_sink_, s.host, s.used);
      return;
    }
    if (cfg_.stage == GpuSinkConfig::Stage::kNone) return;
    ensure_device(cfg_.device);
    // copy, CRC and completion event in one stream's order: no cross-stream wait
    const int64_t t0 = now_ns();
    hip_check(hipMemcpyAsync(dst, s.host, s.used, hipMemcpyHostToDevice, s.st), "hipMemcpyAsync(H2D)");
    const int64_t t1 = now_ns();
    note_hip_call("hipMemcpyAsync(H2D)", s.st_idx, t0, t1);
    if (b) {
      launch_crc32c_batch(*b, d_tables_, s.tiles, s.d_res, s.st);
      note_hip_call("crc launch", s.st_idx, t1, now_ns());
    }
    const int64_t t2 = now_ns();
    hip_check(hipEventRecord(s.ev, s.st), "hipEventRecord");
    note_hip_call("hipEventRecord", s.st_idx, t2, now_ns());
  };
  if (!cfg_.async_submit) {
    s.issued = ++s.posted;
    issue(batch);
    return;
  }
  uint64_t seq;
  {
    std::lock_guard<std::mutex> lk(sub_mu_);
    seq = ++s.posted;
  }
  const bool has = batch != nullptr;
  CrcBatch copy;
  if (has) copy = *batch;
  DeviceSubmitter::get(cfg_.device).post([this, &s, issue, has, copy, seq]() {
    std::string err;
    try {
      issue(has ? &copy : nullptr);
    } catch (const std::exception& e) {
      err = e.what();
    }
    {
      std::lock_guard<std::mutex> lk(sub_mu_);
      s.issued = seq;
      if (!err.empty() && detail_.empty()) {
        mismatch_ = true;
        detail_ = "GPU submit failed: " + err;
      }
    }
    sub_cv_.notify_all();
  });
}

void GpuSink::wait_slot(Slot& s) {
  if (!s.inflight) return;
  RoctxRange rg("gcsb.wait_slot");
  if (cfg_.async_submit) {
    std::unique_lock<std::mutex> lk(sub_mu_);
    sub_cv_.wait(lk, [&] { return s.issued == s.posted; });
  }
  s.inflight = false;
  if (cfg_.stage != GpuSinkConfig::Stage::kH2D) return;  // A/B stages: no GPU work queued
  set_device();
  wait_event(s.ev);
  harvest(s);
}

void GpuSink::wait_event(hipEvent_t ev) {
  if (cfg_.wait_poll_us <= 0) {
    hip_check(hipEventSynchronize(ev), "hipEventSynchronize");
    return;
  }
  // the default 50 us timer slack would stretch every sleep
  static thread_local const bool slack = prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL) == 0;
  (void)slack;
  const timespec ts{0, static_cast<long>(cfg_.wait_poll_us) * 1000L};
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) hip_check(e, "hipEventQuery");
    nanosleep(&ts, nullptr);
  }
}

uint32_t GpuSink::shift(uint32_t v, uint64_t nbytes) {
  if (v == 0 || nbytes == 0) return v;
  for (int i = 0; i < 4; ++i)
    if (op_len_[i] == nbytes) return gf2_multmodp(op_val_[i], v);
  int k = op_rr_++ & 3;
  op_len_[k] = nbytes;
  op_val_[k] = crc32c_x8n(nbytes);
  return gf2_multmodp(op_val_[k], v);
}

void GpuSink::harvest(Slot& s) {
  if (!cfg_.verify) return;
  for (size_t i = 0; i < s.segs.size(); ++i) {
    const SegInfo& g = s.segs[i];
    const volatile CrcSegResult* rv = s.res + i;
    const uint32_t raw = rv->raw;
    const uint32_t status = rv->status;
    obj_raw_ = shift(obj_raw_, g.len) ^ raw;
    obj_len_ += g.len;
    if (g.chunk_start) {
      chunk_raw_ = 0;
      chunk_len_ = 0;
    }
    chunk_raw_ = shift(chunk_raw_, g.len) ^ raw;
    chunk_len_ += g.len;
    if (g.chunk_end && g.has_expected && !g.broken_chunk) {
      any_checked_ = true;
      const uint32_t crc = chunk_raw_ ^ crc32c_fixup(chunk_len_);
      const bool whole = g.chunk_start;
      if (whole) ++stats_.chunks_verified_gpu;
      else ++stats_.chunks_verified_host;
      if (crc != g.expected || (whole && status != 1)) {
        mismatch_ = true;
        char b[160];
        std::snprintf(b, sizeof(b), "chunk crc32c mismatch at offset %llu: got %08x want %08x (gpu status %u)",
                      static_cast<unsigned long long>(g.obj_off + g.len - chunk_len_), crc, g.expected, status);
        detail_ = b;
      }
    }
  }
}

SinkResult GpuSink::finish() {
  RoctxRange rg("gcsb.wait_landed");
  if (cfg_.conn_ring) {
    ring_wait_all();
    ring_fold();
  } else {
    submit_current();
    for (int k = 0; k < cfg_.slots; ++k) wait_slot(slots_[(next_ + k) % cfg_.slots]);
  }
  SinkResult r;
  r.bytes = delivered_;
  r.landed_ns = now_ns();
  if (cfg_.verify && info_.has_crc32c && info_.start_offset == 0 &&
      (info_.size < 0 || static_cast<uint64_t>(info_.size) == obj_len_)) {
    any_checked_ = true;
    ++stats_.objects_verified;
    const uint32_t crc = obj_raw_ ^ crc32c_fixup(obj_len_);
    r.computed_crc32c = crc;
    if (crc != info_.crc32c) {
      mismatch_ = true;
      char b[128];
      std::snprintf(b, sizeof(b), "bad CRC on read: got %08x want %08x", crc, info_.crc32c);
      if (detail_.empty()) detail_ = b;  // keep the first (chunk-level) finding
    }
  } else if (cfg_.verify) {
    r.computed_crc32c = obj_raw_ ^ crc32c_fixup(obj_len_);
  }
  r.verified = any_checked_ && !mismatch_;
  r.crc_mismatch = mismatch_;
  r.detail = detail_;
  return r;
}

void GpuSink::abort() {
  if (cfg_.conn_ring) {
    // its bytes are real (delivered) bytes: let their copies land
    ring_wait_all();
    return;
  }
  if (cur_ >= 0) {
    slots_[cur_].used = 0;
    slots_[cur_].segs.clear();
    cur_ = -1;
  }
  set_device();
  for (Slot& s : slots_)
    if (s.inflight) {
      if (cfg_.async_submit) {  // the hand-off may still be queued on the submitter
        std::unique_lock<std::mutex> lk(sub_mu_);
        sub_cv_.wait(lk, [&] { return s.issued == s.posted; });
      }
      if (cfg_.stage == GpuSinkConfig::Stage::kH2D) hip_check(hipEventSynchronize(s.ev), "hipEventSynchronize");
      s.inflight = false;
    }
}

// ---------------------------------------------------------------------------
// connection ring (engine.h ConnRing): one receive ring per multiplexed
// connection, shared by the sinks of every stream on it

namespace {
// A GPU that never publishes a result (a fault) must not hang the reader or
// a finishing worker forever.
constexpr int64_t kRingWaitLimitNs = 60LL * 1000 * 1000 * 1000;
}  // namespace

ConnRing::ConnRing(int device, size_t slot_bytes, int slots) : device_(device) {
  slot_bytes_ = std::max<size_t>((slot_bytes + 4095) / 4096 * 4096, 65536);
  if (slots < 2) slots = 2;
  res_cap_ = static_cast<size_t>(kMaxSeg);
  ensure_device(device_);
  DeviceStreamPool& pool = DeviceStreamPool::get(device_);
  d_tables_ = device_crc_tables(device_);
  tiles_cap_ = slot_bytes_ / kCrcMinTile + 2 * kMaxSeg + 8;
  d_tiles_ = crc_scratch_alloc(crc_scratch_words(tiles_cap_) * slots);
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&res_host_), sizeof(CrcSegResult) * res_cap_ * slots,
                          hipHostMallocMapped | hipHostMallocCoherent),
            "hipHostMalloc(ring results)");
  std::memset(res_host_, 0, sizeof(CrcSegResult) * res_cap_ * slots);
  const unsigned base = pool.next_base() * static_cast<unsigned>(slots);
  slots_.resize(slots);
  for (int i = 0; i < slots; ++i) {
    RSlot& r = slots_[i];
    r.host = static_cast<uint8_t*>(PinnedPool::get(slot_bytes_, device_numa_node(device_)));
    if (pool.private_streams()) {
      hip_check(hipStreamCreateWithFlags(&r.st, hipStreamNonBlocking), "hipStreamCreate(ring)");
    } else {
      r.st = pool.at(base + static_cast<unsigned>(i));
      r.st_idx = pool.index_of(r.st);
    }
    r.tiles = d_tiles_ + crc_scratch_words(tiles_cap_) * static_cast<size_t>(i);
    r.res = res_host_ + static_cast<size_t>(i) * res_cap_;
    hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&r.d_res), r.res, 0), "hipHostGetDevicePointer");
  }
}

ConnRing::~ConnRing() {
  {
    // every hand-off issued, every launched kernel finished, before the
    // pinned slots and the result block go
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return issued_ == posted_; });
  }
  try {
    ensure_device(device_);
    for (RSlot& r : slots_)
      if (r.submitted > 0) hip_check(hipStreamSynchronize(r.st), "hipStreamSynchronize(ring)");
  } catch (...) {
  }
  for (RSlot& r : slots_) {
    PinnedPool::put(r.host, slot_bytes_);
    if (r.st_idx < 0 && r.st) (void)hipStreamDestroy(r.st);
  }
  if (res_host_) (void)hipHostFree(res_host_);
  if (d_tiles_) (void)hipFree(d_tiles_);
}

ConnRing::Stats ConnRing::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return stats_;
}

// Segments [r.submitted, upto) of slot `slot` to the device submitter: one H2D
// per segment into its object's HBM, then one CRC launch over all of them
// (results at r.res[submitted..upto), published by the kernel).
void ConnRing::submit_locked(int slot, size_t upto) {
  RSlot& r = slots_[slot];
  const size_t a = r.submitted;
  if (upto <= a) return;
  RoctxRange rg("gcsb.ring_submit");
  struct Copy {
    uint8_t* dst;
    const uint8_t* src;
    uint32_t len;
  };
  std::vector<Copy> copies;
  copies.reserve(upto - a);
  // one CRC launch per kMaxSeg segments; the batches run in order on the
  // slot's stream and share its tile scratch
  std::vector<CrcBatch> batches((upto - a + kMaxSeg - 1) / kMaxSeg);
  for (CrcBatch& b : batches) std::memset(&b, 0, sizeof(b));
  for (size_t i = a; i < upto; ++i) {
    const Seg& g = r.segs[i];
    CrcBatch& b = batches[(i - a) / kMaxSeg];
    CrcSeg& c = b.seg[b.nseg++];
    c.addr = g.dst;
    c.len = g.len;
    c.flags = 0;  // chunks are checked by the owner's host fold
    if (g.len) copies.push_back({g.dst, r.host + g.slot_off, g.len});
    __atomic_store_n(&r.res[i].status, kCrcStatusPending, __ATOMIC_RELAXED);
  }
  for (CrcBatch& b : batches) {
    finalize_crc_batch(&b);
    if (b.total_tiles > tiles_cap_) throw std::logic_error("ConnRing: CRC tile scratch too small");
  }
  r.submitted = upto;
  ++stats_.submissions;
  stats_.segments += upto - a;
  ++posted_;
  hipStream_t st = r.st;
  const int st_idx = r.st_idx;
  uint32_t* tiles = r.tiles;
  CrcSegResult* d_res = r.d_res + a;
  CrcSegResult* h_res = r.res + a;
  const int dev = device_;
  const CrcTables* tabs = d_tables_;
  const size_t nres = upto - a;
  DeviceSubmitter::get(device_).post([this, batches, copies, st, st_idx, tiles, d_res, h_res, nres, dev, tabs]() {
    bool ok = true;
    try {
      ensure_device(dev);
      for (const Copy& c : copies) {
        const int64_t t0 = now_ns();
        hip_check(hipMemcpyAsync(c.dst, c.src, c.len, hipMemcpyHostToDevice, st), "hipMemcpyAsync(H2D ring)");
        note_hip_call("hipMemcpyAsync(H2D)", st_idx, t0, now_ns());
      }
      for (size_t k = 0; k < batches.size(); ++k) {
        const int64_t t1 = now_ns();
        launch_crc32c_batch(batches[k], tabs, tiles, d_res + k * kMaxSeg, st);
        note_hip_call("crc launch", st_idx, t1, now_ns());
      }
    } catch (const std::exception&) {
      ok = false;
    }
    std::lock_guard<std::mutex> lk(mu_);
    if (!ok)  // nothing will publish these results: fail them
      for (size_t i = 0; i < nres; ++i) {
        h_res[i].raw = 0;
        __atomic_store_n(&h_res[i].status, 3u, __ATOMIC_RELEASE);
      }
    ++issued_;
    cv_.notify_all();
  });
}

// Copies the results the kernel has published out to their owners, in order.
void ConnRing::collect_locked(RSlot& r) {
  while (r.collected < r.submitted) {
    const CrcSegResult* rv = r.res + r.collected;
    const uint32_t st = __atomic_load_n(&rv->status, __ATOMIC_ACQUIRE);
    if (st == kCrcStatusPending) break;
    const Seg& g = r.segs[r.collected];
    GpuSink::RingRes& o = g.owner->ring_res_[g.seq];
    o.raw = g.len ? rv->raw : 0u;
    o.failed = st == 3u;
    o.done = true;
    if (++g.owner->ring_done_ == g.owner->ring_res_.size() && g.owner->ring_waiting_)
      g.owner->ring_cv_.notify_one();  // that worker's read is complete: wake only it
    ++r.collected;
  }
}

void ConnRing::hand_off_poller_locked() {
  for (GpuSink* w : waiters_)
    if (!owner_done_locked(w)) {
      w->ring_cv_.notify_one();
      return;
    }
}

void ConnRing::collect_all_locked() {
  for (RSlot& r : slots_) collect_locked(r);
}

// Everything the reader is not receiving into goes to the GPU now.
void ConnRing::flush_locked() {
  if (cur_ < 0) return;
  RSlot& r = slots_[cur_];
  size_t upto = r.segs.size();
  if (window_open_ && upto > 0) --upto;
  submit_locked(cur_, upto);
}

// The reader's next slot: every result of its last use collected first.
ConnRing::RSlot& ConnRing::take_slot_locked(std::unique_lock<std::mutex>& lk) {
  if (cur_ >= 0) {
    RSlot& old = slots_[cur_];
    submit_locked(cur_, old.segs.size());
    old.filling = false;
    cur_ = -1;
    ++stats_.slots_filled;
  }
  RSlot& r = slots_[next_];
  collect_locked(r);
  if (r.collected < r.segs.size()) {
    ++stats_.reader_waits;
    const int64_t t0 = now_ns();
    const timespec ts{0, 10000};
    while (r.collected < r.segs.size()) {
      if (now_ns() - t0 > kRingWaitLimitNs)
        throw std::runtime_error("connection ring: a slot's CRC results did not arrive within 60 s");
      lk.unlock();
      nanosleep(&ts, nullptr);
      lk.lock();
      collect_locked(r);
    }
    stats_.reader_wait_s += (now_ns() - t0) / 1e9;
  }
  r.segs.clear();
  r.used = 0;
  r.submitted = r.collected = 0;
  r.filling = true;
  ++r.gen;
  cur_ = next_;
  next_ = (next_ + 1) % static_cast<int>(slots_.size());
  return r;
}

bool GpuSink::ring_extends(const ConnRing& R) const {
  if (R.cur_ < 0 || ring_open_slot_ != R.cur_) return false;
  const ConnRing::RSlot& r = R.slots_[R.cur_];
  return ring_open_gen_ == r.gen && ring_open_seg_ + 1 == r.segs.size() && ring_open_seg_ >= r.submitted &&
         r.segs[ring_open_seg_].owner == this;
}

Window GpuSink::ring_acquire() {
  ConnRing& R = *cfg_.conn_ring;
  if (delivered_ >= obj_cap_)
    // size unknown so far (or larger than announced): grow, keeping landed bytes
    grow_object_buffer(std::max<uint64_t>(2 * obj_cap_, delivered_ + R.slot_bytes_));
  std::unique_lock<std::mutex> lk(R.mu_);
  R.window_open_ = false;  // a window the reader never committed (its recv failed) is dropped
  R.window_owner_ = nullptr;
  ConnRing::RSlot* r = R.cur_ >= 0 ? &R.slots_[R.cur_] : nullptr;
  const bool mine = r && ring_extends(R);
  if (!r || r->used == R.slot_bytes_ || (!mine && r->segs.size() >= static_cast<size_t>(kMaxSeg))) {
    r = &R.take_slot_locked(lk);
    ring_open_slot_ = -1;
  }
  if (!ring_extends(R)) {
    ConnRing::Seg g;
    g.owner = this;
    g.seq = ring_res_.size();
    g.slot_off = static_cast<uint32_t>(r->used);
    g.dst = obj_dst_ + delivered_;
    RingRes rr;
    rr.obj_off = delivered_;
    ring_res_.push_back(rr);
    r->segs.push_back(g);
    ring_open_slot_ = R.cur_;
    ring_open_seg_ = r->segs.size() - 1;
    ring_open_gen_ = r->gen;
  }
  size_t cap = R.slot_bytes_ - r->used;
  if (obj_cap_ - delivered_ < cap) cap = obj_cap_ - delivered_;
  R.window_open_ = true;
  R.window_owner_ = this;
  return Window{r->host + r->used, cap};
}

void GpuSink::ring_commit(size_t n) {
  ConnRing& R = *cfg_.conn_ring;
  std::lock_guard<std::mutex> lk(R.mu_);
  R.window_open_ = false;
  R.window_owner_ = nullptr;
  if (ring_open_slot_ != R.cur_ || R.cur_ < 0) throw std::logic_error("GpuSink::commit outside an acquired window");
  ConnRing::RSlot& r = R.slots_[R.cur_];
  ConnRing::Seg& g = r.segs[ring_open_seg_];
  g.len += static_cast<uint32_t>(n);
  r.used += n;
  ring_res_[g.seq].len += static_cast<uint32_t>(n);
  delivered_ += n;
}

// Submits what the reader is not writing into and waits for every segment
// of this sink to have its result (the kernel publishes them; no HIP call).
void GpuSink::ring_wait_all() {
  ConnRing& R = *cfg_.conn_ring;
  std::unique_lock<std::mutex> lk(R.mu_);
  // this read is over (finish / abort / a retry): a window the reader opened
  // for it and never committed (its recv failed) will never be written
  if (R.window_open_ && R.window_owner_ == this) R.window_open_ = false;
  if (R.owner_done_locked(this)) return;
  R.flush_locked();
  R.collect_all_locked();
  if (R.owner_done_locked(this)) {
    ring_open_slot_ = -1;
    return;
  }
  // One finishing worker at a time polls the kernel's host-visible status
  // words (no HIP call) and collects for everyone; the others sleep on their
  // own condition variable until a collect completes their read or the
  // poller role is handed to them.  Before: every one of up to 48 finishing
  // workers woke each 10 us and took mu_, which the connection's reader
  // takes twice per recv.
  const timespec ts{0, 10000};
  const int64_t t0 = now_ns();
  ring_waiting_ = true;
  R.waiters_.push_back(this);
  struct Leave {
    ConnRing& R;
    GpuSink* me;
    ~Leave() {
      me->ring_waiting_ = false;
      auto it = std::find(R.waiters_.begin(), R.waiters_.end(), me);
      if (it != R.waiters_.end()) R.waiters_.erase(it);
    }
  } leave{R, this};
  while (!R.owner_done_locked(this)) {
    if (now_ns() - t0 > kRingWaitLimitNs)
      throw std::runtime_error("connection ring: this read's CRC results did not arrive within 60 s");
    if (R.poller_) {
      ++R.stats_.finish_sleeps;
      // bounded: a lost hand-off costs one period, not the read
      ring_cv_.wait_for(lk, std::chrono::milliseconds(1));
      continue;
    }
    R.poller_ = true;
    lk.unlock();
    nanosleep(&ts, nullptr);
    lk.lock();
    R.poller_ = false;
    ++R.stats_.finish_polls;
    // a segment still being written (the reader's open window) is never this
    // sink's once its read ended; anything else unsubmitted goes now
    R.flush_locked();
    R.collect_all_locked();
  }
  ring_open_slot_ = -1;
  R.hand_off_poller_locked();  // still under mu_: the next waiter polls
}

// Host fold of this read's segment CRCs: every chunk (gRPC message) against
// its checksum, and the object.
void GpuSink::ring_fold() {
  std::lock_guard<std::mutex> lk(cfg_.conn_ring->mu_);
  size_t ci = 0;
  for (const RingRes& g : ring_res_) {
    if (g.failed && detail_.empty()) {
      mismatch_ = true;
      detail_ = "GPU submit failed (connection ring)";
    }
    obj_raw_ = shift(obj_raw_, g.len) ^ g.raw;
    obj_len_ += g.len;
    while (ci < chunks_.size() && chunks_[ci].closed && chunks_[ci].end <= g.obj_off) ++ci;
    if (ci >= chunks_.size()) continue;
    ChunkMark& m = chunks_[ci];
    if (g.obj_off == m.start) {
      chunk_raw_ = 0;
      chunk_len_ = 0;
    }
    if (g.obj_off < m.start) continue;  // bytes outside any chunk
    chunk_raw_ = shift(chunk_raw_, g.len) ^ g.raw;
    chunk_len_ += g.len;
    if (m.closed && g.obj_off + g.len == m.end) {
      if (m.has_crc && !m.broken) {
        any_checked_ = true;
        ++stats_.chunks_verified_host;
        const uint32_t crc = chunk_raw_ ^ crc32c_fixup(chunk_len_);
        if (crc != m.crc) {
          mismatch_ = true;
          char b[160];
          std::snprintf(b, sizeof(b), "chunk crc32c mismatch at offset %llu: got %08x want %08x",
                        static_cast<unsigned long long>(m.start), crc, m.crc);
          detail_ = b;
        }
      }
      ++ci;
    }
  }
  stats_.segments += ring_res_.size();
}

// ---------------------------------------------------------------------------
// write path: HBM -> pinned ring (D2H) -> transport

namespace {
// Per-device pool of CRC tile scratch + host-mapped result blocks for the
// upload sources (one per staging slot): a source lives for one upload, and
// hipMalloc / hipHostMalloc per upload would cost more than its CRCs.
struct CrcScratchBlock {
  uint32_t* tiles = nullptr;
  size_t tiles_cap = 0;
  CrcSegResult* res = nullptr;
  CrcSegResult* d_res = nullptr;
};
std::mutex g_crc_pool_mu;
std::map<int, std::vector<CrcScratchBlock>> g_crc_pool;

CrcScratchBlock crc_block_get(int device, size_t tiles_cap) {
  {
    std::lock_guard<std::mutex> lk(g_crc_pool_mu);
    auto& v = g_crc_pool[device];
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i].tiles_cap >= tiles_cap) {
        CrcScratchBlock b = v[i];
        v.erase(v.begin() + static_cast<long>(i));
        return b;
      }
  }
  CrcScratchBlock b;
  b.tiles_cap = tiles_cap;
  b.tiles = crc_scratch_alloc(tiles_cap);
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&b.res), sizeof(CrcSegResult) * kMaxSeg,
                          hipHostMallocMapped | hipHostMallocCoherent),
            "hipHostMalloc(upload CRC results)");
  std::memset(b.res, 0, sizeof(CrcSegResult) * kMaxSeg);
  hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&b.d_res), b.res, 0), "hipHostGetDevicePointer");
  return b;
}

void crc_block_put(int device, const CrcScratchBlock& b) {
  std::lock_guard<std::mutex> lk(g_crc_pool_mu);
  auto& v = g_crc_pool[device];
  if (v.size() < 64) {
    v.push_back(b);
    return;
  }
  (void)hipFree(b.tiles);
  (void)hipHostFree(b.res);
}
}  // namespace

GpuByteSource::GpuByteSource(int device, const void* dptr, uint64_t n, size_t slot_bytes, int slots, bool gpu_crc,
                             bool async_stage)
    : device_(device),
      src_(static_cast<const uint8_t*>(dptr)),
      n_(n),
      // a ring slot never larger than the (part of the) object it stages
      slot_bytes_(std::max<size_t>(std::min<uint64_t>(slot_bytes, (n + 65535) / 65536 * 65536), 65536)),
      nslots_(std::max(2, slots)) {
  async_stage_ = async_stage;
  if (n_ <= kWholeRingMax)
    nslots_ = std::max<int>(nslots_, static_cast<int>((n_ + slot_bytes_ - 1) / slot_bytes_));
  hip_check(hipSetDevice(device_), "hipSetDevice");
  DeviceStreamPool& pool = DeviceStreamPool::get(device_);
  // The staging copies go round-robin over 2 pool streams, not one per slot,
  // and the same 2 for every source:
  // after a device-wide synchronize (the bench's torch.cuda.synchronize()
  // around every timed region) the first D2H hipMemcpyAsync on one of the
  // further streams blocked ~7 ms -- the first timed upload's 13.6 ms p99.
  // With 2 streams: first upload 6.1 ms, p99 6.3
  // (scripts/experiments/write_tail.py --gap sync; profiles/r2_write).
  constexpr unsigned nst = 2;
  // every upload source of the process shares the same nst streams: the 8
  // parts of a parallel composite upload spread over all 8 pool streams had
  // their first upload after the sync at 10.3 ms vs p50 2.7
  // (profiles/r2_final_s4 rank0_slowest)
  const unsigned base = 0;
  if (pool.private_streams())
    hip_check(hipStreamCreateWithFlags(&own_stream_, hipStreamNonBlocking), "hipStreamCreate");
  st_.resize(nslots_);
  st_idx_.assign(nslots_, -1);
  for (int i = 0; i < nslots_; ++i) {
    st_[i] = own_stream_ ? own_stream_ : pool.at(base + static_cast<unsigned>(i) % nst);
    if (!own_stream_) st_idx_[i] = pool.index_of(st_[i]);
  }
  host_.resize(nslots_);
  ev_.resize(nslots_);
  slot_off_.assign(nslots_, ~0ull);
  slot_len_.assign(nslots_, 0);
  for (int i = 0; i < nslots_; ++i) {
    host_[i] = static_cast<uint8_t*>(PinnedPool::get(slot_bytes_, device_numa_node(device_)));
    ev_[i] = EventPool::get(device_);
  }
  if (gpu_crc) {
    // Chunk CRCs on a grid that the transport's upload messages fall on:
    // messages are <= 2 MiB (gRPC MAX_WRITE_CHUNK_BYTES) and never cross a
    // staging slot, so with slot-aligned slots gcd(slot, 2 MiB) tiles them.
    const uint64_t g = std::gcd<uint64_t>(slot_bytes_, uint64_t(2) << 20);
    grid_ = g >= 65536 ? g : 0;
    chunk_ = grid_ ? grid_ : slot_bytes_;
    if ((slot_bytes_ + chunk_ - 1) / chunk_ > static_cast<uint64_t>(kMaxSeg)) {  // one launch per slot
      grid_ = 0;
      chunk_ = slot_bytes_;
    }
    const size_t nchunks = static_cast<size_t>((n_ + chunk_ - 1) / chunk_);
    chunk_crc_.assign(nchunks, 0);
    chunk_known_.assign(nchunks, 0);
    d_tables_ = device_crc_tables(device_);
    scr_.resize(nslots_);
    for (int i = 0; i < nslots_; ++i) {
      CrcScratchBlock b = crc_block_get(device_, slot_bytes_ / kCrcMinTile + 2 * kMaxSeg + 8);
      scr_[i] = {b.tiles, b.tiles_cap, b.res, b.d_res};
    }
    has_crc_ = true;
  }
  slot_harvested_.assign(nslots_, 1);
  restart(0);
}

bool GpuByteSource::range_crc32c(uint64_t off, size_t len, uint32_t* crc) {
  if (grid_ == 0 || len == 0 || off % grid_ != 0) return false;
  const uint64_t end = off + len;
  if (end > n_ || (end % grid_ != 0 && end != n_)) return false;
  const size_t i = off / grid_, j = (end + grid_ - 1) / grid_;
  if (j > chunk_crc_.size()) return false;
  for (size_t k = i; k < j; ++k)
    if (!chunk_known_[k]) return false;  // not staged yet: the caller checksums the bytes
  uint32_t c = chunk_crc_[i];
  for (size_t k = i + 1; k < j; ++k) c = crc32c_combine(c, chunk_crc_[k], std::min<uint64_t>(grid_, n_ - k * grid_));
  *crc = c;
  ++range_hits_;
  return true;
}

void GpuByteSource::harvest(int slot) const {
  if (slot_harvested_[slot] || !has_crc_ || slot_off_[slot] == ~0ull) return;
  slot_harvested_[slot] = 1;
  const uint64_t off = slot_off_[slot];
  const size_t nseg = static_cast<size_t>((slot_len_[slot] + chunk_ - 1) / chunk_);
  for (size_t k = 0; k < nseg; ++k) {
    const CrcSegResult& r = scr_[slot].res[k];
    if (__atomic_load_n(&r.status, __ATOMIC_ACQUIRE) == kCrcStatusPending)
      throw std::logic_error("GpuByteSource: a staged slot's CRC result is missing");
    const size_t c = static_cast<size_t>(off / chunk_) + k;
    if (!chunk_known_[c]) {
      chunk_known_[c] = 1;
      ++chunks_known_;
    }
    chunk_crc_[c] = r.crc;
  }
}

bool GpuByteSource::crc32c_ready() const { return has_crc_ && (crc_done_ || chunks_known_ == chunk_crc_.size()); }

uint32_t GpuByteSource::crc32c() const {
  if (!has_crc_) return 0;
  if (crc_done_) return crc_;
  if (chunks_known_ < chunk_crc_.size()) {
    await_async();
    // asked before the upload staged every slot: collect what is in flight
    for (int i = 0; i < nslots_; ++i)
      if (!slot_harvested_[i] && slot_off_[i] != ~0ull) {
        hip_check(hipEventSynchronize(ev_[i]), "hipEventSynchronize");
        harvest(i);
      }
  }
  if (chunks_known_ == chunk_crc_.size()) {
    uint32_t c = 0;
    for (size_t k = 0; k < chunk_crc_.size(); ++k)
      c = k ? crc32c_combine(c, chunk_crc_[k], std::min<uint64_t>(chunk_, n_ - k * chunk_)) : chunk_crc_[0];
    crc_ = n_ ? c : 0;
  } else {
    // an object larger than the staging ring, asked for up front: one
    // whole-object pass now
    crc_ = gpu_crc32c(device_, src_, n_);
  }
  crc_done_ = true;
  return crc_;
}

GpuByteSource::~GpuByteSource() {
  try {
    wait_all();
  } catch (...) {
  }
  for (int i = 0; i < nslots_; ++i) {
    PinnedPool::put(host_[i], slot_bytes_);
    EventPool::put(device_, ev_[i]);
  }
  for (const SlotCrc& c : scr_) crc_block_put(device_, {c.tiles, c.tiles_cap, c.res, c.d_res});
  if (own_stream_) (void)hipStreamDestroy(own_stream_);
}

void GpuByteSource::await_async() const {
  std::unique_lock<std::mutex> lk(amu_);
  acv_.wait(lk, [&] { return !async_busy_; });
}

void GpuByteSource::await_issued(int slot) const {
  if (issued_.load(std::memory_order_acquire) > slot) return;
  std::unique_lock<std::mutex> lk(amu_);
  acv_.wait(lk, [&] { return issued_.load(std::memory_order_acquire) > slot || !async_busy_; });
  if (!async_err_.empty()) throw std::runtime_error("GpuByteSource: staging on the submitter: " + async_err_);
}

// This source's queued copies (its slot events; the pool streams are shared).
void GpuByteSource::wait_all() {
  await_async();
  hip_check(hipSetDevice(device_), "hipSetDevice");
  for (int i = 0; i < nslots_; ++i)
    if (slot_off_[i] != ~0ull) {
      hip_check(hipEventSynchronize(ev_[i]), "hipEventSynchronize");
      harvest(i);
    }
}

void GpuByteSource::issue(int slot, uint64_t off) {
  size_t len = static_cast<size_t>(std::min<uint64_t>(slot_bytes_, n_ - off));
  slot_off_[slot] = off;
  slot_len_[slot] = len;
  const int64_t t0 = now_ns();
  hip_check(hipMemcpyAsync(host_[slot], src_ + off, len, hipMemcpyDeviceToHost, st_[slot]), "hipMemcpyAsync(D2H)");
  const int64_t t1 = now_ns();
  note_hip_call("hipMemcpyAsync(D2H)", st_idx_[slot], t0, t1);
  if (has_crc_) {
    // the slot's chunk CRCs from HBM, on the copy's stream (both only read
    // the object): ready with the slot's event
    CrcBatch b;
    std::memset(&b, 0, sizeof(b));
    for (uint64_t o = off; o < off + len; o += chunk_) {
      CrcSeg& c = b.seg[b.nseg++];
      c.addr = src_ + o;
      c.len = static_cast<uint32_t>(std::min<uint64_t>(chunk_, off + len - o));
      c.flags = 0;
    }
    finalize_crc_batch(&b);
    if (b.total_tiles > scr_[slot].tiles_cap) throw std::logic_error("GpuByteSource: CRC tile scratch too small");
    for (uint32_t k = 0; k < b.nseg; ++k) __atomic_store_n(&scr_[slot].res[k].status, kCrcStatusPending, __ATOMIC_RELAXED);
    launch_crc32c_batch(b, d_tables_, scr_[slot].tiles, scr_[slot].d_res, st_[slot]);
    slot_harvested_[slot] = 0;
    note_hip_call("crc launch(upload)", st_idx_[slot], t1, now_ns());
  }
  const int64_t t2 = now_ns();
  hip_check(hipEventRecord(ev_[slot], st_[slot]), "hipEventRecord");
  note_hip_call("hipEventRecord(D2H)", st_idx_[slot], t2, now_ns());
  copies_.fetch_add(1, std::memory_order_relaxed);
}

void GpuByteSource::restart(uint64_t off) {
  wait_all();
  pos_ = off;
  uint64_t base = off / slot_bytes_ * slot_bytes_;
  next_issue_ = base;
  cur_ = 0;
  slot_off_.assign(nslots_, ~0ull);
  async_err_.clear();
  // the whole object in one ring, staged from its start: no slot is ever
  // refilled, so the submitter can issue every slot past the first few
  // while this thread already sends (next() waits per slot on issued_)
  const bool whole = async_stage_ && base == 0 && stable_until_done() && nslots_ > kSyncSlots;
  int i = 0;
  for (; i < nslots_ && next_issue_ < n_ && (!whole || i < kSyncSlots); ++i) {
    issue(i, next_issue_);
    next_issue_ += slot_bytes_;
  }
  if (!whole || next_issue_ >= n_) {
    issued_.store(nslots_, std::memory_order_release);
    return;
  }
  issued_.store(i, std::memory_order_release);
  {
    std::lock_guard<std::mutex> lk(amu_);
    async_busy_ = true;
  }
  const int first = i;
  const uint64_t from = next_issue_;
  next_issue_ = n_;  // every slot is (being) issued
  DeviceSubmitter::get(device_).post([this, first, from] {
    std::string err;
    try {
      uint64_t o = from;
      for (int s = first; s < nslots_ && o < n_; ++s, o += slot_bytes_) {
        issue(s, o);
        issued_.store(s + 1, std::memory_order_release);
        { std::lock_guard<std::mutex> lk(amu_); }  // a waiter between its check and its wait sees this
        acv_.notify_all();
      }
    } catch (const std::exception& e) {
      err = e.what();
    }
    std::lock_guard<std::mutex> lk(amu_);
    async_err_ = err;
    async_busy_ = false;
    issued_.store(err.empty() ? nslots_ : issued_.load(), std::memory_order_release);
    acv_.notify_all();
  });
}

void GpuByteSource::seek(uint64_t off) {
  if (off == pos_) return;
  restart(off);
}

std::pair<const uint8_t*, size_t> GpuByteSource::next(size_t max) {
  if (pos_ >= n_ || max == 0) return {nullptr, 0};
  const int64_t w0 = now_ns();
  await_issued(cur_);
  // slot cur_ holds [slot_off_, slot_off_ + len) and pos_ lies inside it
  if (slot_off_[cur_] == ~0ull || pos_ >= slot_off_[cur_] + slot_len_[cur_]) {
    // the consumer moved past this slot: refill it far ahead, advance
    if (slot_off_[cur_] != ~0ull && next_issue_ < n_) {
      issue(cur_, next_issue_);
      next_issue_ += slot_bytes_;
    }
    cur_ = (cur_ + 1) % nslots_;
    await_issued(cur_);
  }
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipEventSynchronize(ev_[cur_]), "hipEventSynchronize");
  stage_wait_ns_ += now_ns() - w0;
  harvest(cur_);
  const uint64_t so = slot_off_[cur_];
  if (so == ~0ull || pos_ < so || pos_ >= so + slot_len_[cur_])
    throw std::logic_error("GpuByteSource: staging ring out of step");
  size_t k = static_cast<size_t>(std::min<uint64_t>(max, so + slot_len_[cur_] - pos_));
  const uint8_t* p = host_[cur_] + (pos_ - so);
  pos_ += k;
  return {p, k};
}

// ---------------------------------------------------------------------------
// utilities

DeviceBuffer::~DeviceBuffer() {
  if (p_) {
    (void)hipSetDevice(device_);
    (void)hipFree(p_);
  }
}

uint8_t* DeviceBuffer::ensure(size_t n) {
  if (n <= cap_ && p_) return p_;
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  if (p_) hip_check(hipFree(p_), "hipFree");
  p_ = nullptr;
  size_t cap = std::max<size_t>((n + (2u << 20) - 1) / (2u << 20) * (2u << 20), 2u << 20);
  hip_check(hipMalloc(reinterpret_cast<void**>(&p_), cap), "hipMalloc(landing)");
  cap_ = cap;
  return p_;
}

uint32_t gpu_crc32c(int device, const void* dptr, size_t n, size_t chunk, std::vector<uint32_t>* chunks) {
  if (n == 0) return 0;
  hip_check(hipSetDevice(device), "hipSetDevice");
  const CrcTables* tabs = device_crc_tables(device);
  DeviceCtx& c = device_ctx(device);
  std::lock_guard<std::mutex> lk(c.mu);
  // kMaxSeg segments per batch (>= 1 MiB, 4 KiB multiples): K1 covers every
  // tile in parallel and K2 folds with kMaxSeg workgroups, not one.
  size_t seg = (n + kMaxSeg - 1) / kMaxSeg;
  seg = std::min<size_t>(std::max<size_t>((seg + kCrcRoundBytes - 1) / kCrcRoundBytes * kCrcRoundBytes, 1u << 20),
                         1u << 30);
  if (chunk > 0) {
    seg = std::min<size_t>(chunk, 1u << 30);
    if (chunks) chunks->reserve(chunks->size() + (n + seg - 1) / seg);
  }
  const uint8_t* p = static_cast<const uint8_t*>(dptr);
  uint32_t crc = 0;
  size_t off = 0;
  while (off < n) {
    CrcBatch b;
    std::memset(&b, 0, sizeof(b));
    while (off < n && b.nseg < static_cast<uint32_t>(kMaxSeg)) {
      size_t len = std::min(seg, n - off);
      b.seg[b.nseg].addr = p + off;
      b.seg[b.nseg].len = static_cast<uint32_t>(len);
      ++b.nseg;
      off += len;
    }
    finalize_crc_batch(&b);
    if (b.total_tiles + 1 > c.tiles_cap || !c.d_tiles) {
      if (c.d_tiles) (void)hipFree(c.d_tiles);
      c.tiles_cap = b.total_tiles + 1;
      c.d_tiles = crc_scratch_alloc(c.tiles_cap);
    }
    launch_crc32c_batch(b, tabs, c.d_tiles, c.d_res, c.st);
    hip_check(hipStreamSynchronize(c.st), "hipStreamSynchronize");
    for (uint32_t i = 0; i < b.nseg; ++i) {
      crc = crc32c_combine(crc, c.res[i].crc, b.seg[i].len);
      if (chunks) chunks->push_back(c.res[i].crc);
    }
  }
  return crc;
}

double gpu_crc32c_throughput(int device, const void* dptr, size_t n, int iters, size_t seg_bytes, uint32_t* raw0,
                             int tile_log2, uint32_t probe) {
  hip_check(hipSetDevice(device), "hipSetDevice");
  const CrcTables* tabs = device_crc_tables(device);
  hipStream_t st;
  hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
  // one batch of up to kMaxSeg segments covering [dptr, dptr+n)
  CrcBatch b;
  std::memset(&b, 0, sizeof(b));
  const uint8_t* p = static_cast<const uint8_t*>(dptr);
  size_t off = 0;
  while (off < n && b.nseg < static_cast<uint32_t>(kMaxSeg)) {
    size_t len = std::min(seg_bytes, n - off);
    b.seg[b.nseg].addr = p + off;
    b.seg[b.nseg].len = static_cast<uint32_t>(len);
    ++b.nseg;
    off += len;
  }
  finalize_crc_batch(&b, static_cast<uint32_t>(tile_log2));
  b.probe = probe;
  uint32_t* d_tiles = crc_scratch_alloc(b.total_tiles + 1);
  CrcSegResult* res = nullptr;
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&res), sizeof(CrcSegResult) * kMaxSeg,
                          hipHostMallocMapped | hipHostMallocCoherent),
            "hipHostMalloc");
  CrcSegResult* d_res = nullptr;
  hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_res), res, 0), "hipHostGetDevicePointer");
  hipEvent_t e0, e1;
  hip_check(hipEventCreate(&e0), "hipEventCreate");
  hip_check(hipEventCreate(&e1), "hipEventCreate");
  launch_crc32c_batch(b, tabs, d_tiles, d_res, st);  // warm-up
  hip_check(hipEventRecord(e0, st), "hipEventRecord");
  for (int i = 0; i < iters; ++i) launch_crc32c_batch(b, tabs, d_tiles, d_res, st);
  hip_check(hipEventRecord(e1, st), "hipEventRecord");
  hip_check(hipEventSynchronize(e1), "hipEventSynchronize");
  float ms = 0;
  hip_check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
  if (raw0) *raw0 = res[0].crc;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(d_tiles);
  (void)hipHostFree(res);
  (void)hipStreamDestroy(st);
  return static_cast<double>(off) * iters / (ms / 1e3) / 1e9;  // GB/s over the covered bytes
}

void gpu_fill_pattern(int device, void* dptr, uint64_t n, uint64_t rot, uint64_t obj_off) {
  hip_check(hipSetDevice(device), "hipSetDevice");
  launch_fill_pattern(static_cast<uint8_t*>(dptr), n, rot, obj_off, nullptr);
  hip_check(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
}

uint64_t gpu_verify_pattern(int device, const void* dptr, uint64_t n, uint64_t rot, uint64_t obj_off,
                            uint64_t* first_bad) {
  hip_check(hipSetDevice(device), "hipSetDevice");
  unsigned long long* d = nullptr;
  hip_check(hipMalloc(reinterpret_cast<void**>(&d), 16), "hipMalloc");
  unsigned long long init[2] = {0ull, ~0ull};
  hip_check(hipMemcpy(d, init, 16, hipMemcpyHostToDevice), "hipMemcpy");
  launch_verify_pattern(static_cast<const uint8_t*>(dptr), n, rot, obj_off, d, d + 1, nullptr);
  unsigned long long out[2];
  hip_check(hipMemcpy(out, d, 16, hipMemcpyDeviceToHost), "hipMemcpy");
  (void)hipFree(d);
  if (first_bad) *first_bad = out[1];
  return out[0];
}

}  // namespace gcsb
