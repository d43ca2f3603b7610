#include "core/affinity.h"

#include <pthread.h>
#include <sched.h>

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

void name_current_thread(const char* name) {
  char buf[16];
  std::snprintf(buf, sizeof(buf), "%s", name);
  pthread_setname_np(pthread_self(), buf);
}

std::vector<int> cpus_for(const std::vector<int>& cpus, int k, bool spread) {
  if (cpus.empty() || !spread) return cpus;
  return {cpus[static_cast<size_t>(k) % cpus.size()]};
}

}  // namespace gcsb
