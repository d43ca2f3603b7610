#include "core/affinity.h"
#include "core/sched_probe.h"

#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "core/util.h"

namespace gcsb {

std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  for (auto part : split(trim(s), ',')) {
    part = trim(part);
    if (part.empty()) continue;
    size_t dash = part.find('-');
    if (dash == std::string_view::npos) {
      out.push_back(std::atoi(std::string(part).c_str()));
    } else {
      int a = std::atoi(std::string(part.substr(0, dash)).c_str());
      int b = std::atoi(std::string(part.substr(dash + 1)).c_str());
      for (int c = a; c <= b; ++c) out.push_back(c);
    }
  }
  return out;
}

bool pin_current_thread(const std::vector<int>& cpus) {
  if (cpus.empty()) return true;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  return pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0;
}

std::vector<long> numa_nodes_of(const void* p, size_t len, size_t stride) {
  std::vector<long> counts(kNumaMaxNodes + 1, 0);
  if (!p || len == 0) return counts;
  stride = std::max<size_t>(stride, 4096);
  const uintptr_t base = reinterpret_cast<uintptr_t>(p) & ~uintptr_t(4095);
  const uintptr_t end = reinterpret_cast<uintptr_t>(p) + len;
  std::vector<void*> pages;
  for (uintptr_t a = base; a < end; a += stride) pages.push_back(reinterpret_cast<void*>(a));
  std::vector<int> status(pages.size(), -1);
  long rc = ::syscall(SYS_move_pages, 0, pages.size(), pages.data(), nullptr, status.data(), 0);
  for (int st : status) {
    if (rc == 0 && st >= 0 && st < kNumaMaxNodes) ++counts[st];
    else ++counts[kNumaAbsent];
  }
  return counts;
}

int current_numa_node() {
  unsigned cpu = 0, node = 0;
  if (::syscall(SYS_getcpu, &cpu, &node, nullptr) != 0) return -1;
  return static_cast<int>(node);
}

bool prefer_numa_node(int node) {
  constexpr int kMpolDefault = 0, kMpolPreferred = 1;
  if (node < 0 || node >= 64) return ::syscall(SYS_set_mempolicy, kMpolDefault, nullptr, 0) == 0;
  unsigned long mask = 1ul << node;
  return ::syscall(SYS_set_mempolicy, kMpolPreferred, &mask, 64) == 0;
}

bool bind_numa_node(int node) {
  constexpr int kMpolDefault = 0, kMpolBind = 2;
  if (node < 0 || node >= 64) return ::syscall(SYS_set_mempolicy, kMpolDefault, nullptr, 0) == 0;
  unsigned long mask = 1ul << node;
  return ::syscall(SYS_set_mempolicy, kMpolBind, &mask, 64) == 0;
}

bool bind_range_to_node(void* p, size_t len, int node) {
  constexpr int kMpolBind = 2;
  if (node < 0 || node >= 64) return false;
  unsigned long mask = 1ul << node;
  return ::syscall(SYS_mbind, p, len, kMpolBind, &mask, 64, 0) == 0;
}

void name_current_thread(const char* name) {
  char buf[16];
  std::snprintf(buf, sizeof(buf), "%s", name);
  pthread_setname_np(pthread_self(), buf);
  register_named_thread(buf);  // core/sched_probe.h
}

std::vector<int> cpus_for(const std::vector<int>& cpus, int k, bool spread) {
  if (cpus.empty() || !spread) return cpus;
  return {cpus[static_cast<size_t>(k) % cpus.size()]};
}

}  // namespace gcsb
