#include "core/hugebuf.h"

#include <sys/mman.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>
#include <new>

namespace gcsb {

uint8_t* huge_alloc(size_t n) {
  const size_t huge = size_t(2) << 20;
  const size_t len = huge_round(n ? n : 1);
  // over-map by one huge page and trim, for 2 MiB alignment
  void* raw = ::mmap(nullptr, len + huge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (raw == MAP_FAILED) throw std::bad_alloc();
  const uintptr_t a = (reinterpret_cast<uintptr_t>(raw) + huge - 1) & ~(huge - 1);
  const size_t head = a - reinterpret_cast<uintptr_t>(raw);
  if (head) ::munmap(raw, head);
  if (huge - head) ::munmap(reinterpret_cast<void*>(a + len), huge - head);
  void* p = reinterpret_cast<void*>(a);
  (void)::madvise(p, len, MADV_HUGEPAGE);
  std::memset(p, 0, len);  // fault in now, not inside a timed read
  return static_cast<uint8_t*>(p);
}

void huge_free(void* p, size_t n) {
  if (p) ::munmap(p, huge_round(n ? n : 1));
}

namespace {
std::mutex& pool_mu() {
  static std::mutex m;
  return m;
}
std::map<size_t, std::vector<uint8_t*>>& pool() {
  static auto* f = new std::map<size_t, std::vector<uint8_t*>>();  // outlives every user
  return *f;
}
size_t& pool_bytes() {
  static size_t b = 0;
  return b;
}
constexpr size_t kPoolMax = size_t(1) << 30;
}  // namespace

long long thp_bytes_of(const void* p, size_t len) {
  FILE* f = std::fopen("/proc/self/smaps", "r");
  if (!f) return -1;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p), b = a + len;
  char line[512];
  bool in = false;
  uintptr_t lo = 0, hi = 0;
  long long total = 0;
  while (std::fgets(line, sizeof(line), f)) {
    unsigned long s = 0, e = 0;
    if (std::sscanf(line, "%lx-%lx ", &s, &e) == 2 && std::strchr(line, '-') < std::strchr(line, ' ')) {
      lo = s, hi = e;
      in = hi > a && lo < b;
      continue;
    }
    long long kb = 0;
    if (in && std::sscanf(line, "AnonHugePages: %lld kB", &kb) == 1) {
      const uintptr_t ov = std::min(hi, b) - std::max(lo, a);
      total += std::min<long long>(kb * 1024, static_cast<long long>(ov));
    }
  }
  std::fclose(f);
  return total;
}

uint8_t* huge_take(size_t n) {
  const size_t r = huge_round(n ? n : 1);
  {
    std::lock_guard<std::mutex> lk(pool_mu());
    auto& v = pool()[r];
    if (!v.empty()) {
      uint8_t* p = v.back();
      v.pop_back();
      pool_bytes() -= r;
      return p;
    }
  }
  return huge_alloc(r);
}

void huge_give(void* p, size_t n) {
  if (!p) return;
  const size_t r = huge_round(n ? n : 1);
  {
    std::lock_guard<std::mutex> lk(pool_mu());
    if (pool_bytes() + r <= kPoolMax) {
      pool()[r].push_back(static_cast<uint8_t*>(p));
      pool_bytes() += r;
      return;
    }
  }
  huge_free(p, r);
}

}  // namespace gcsb
