#include "core/sched_probe.h"

#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <time.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <set>

namespace gcsb {

namespace {
std::mutex g_mu;
std::map<int, std::string>& registry() {
  static auto* r = new std::map<int, std::string>();  // process lifetime
  return *r;
}

// Whole small /proc file into buf (NUL-terminated); false if unreadable.
bool read_small(const char* path, char* buf, size_t cap) {
  FILE* f = std::fopen(path, "r");
  if (!f) return false;
  const size_t n = std::fread(buf, 1, cap - 1, f);
  std::fclose(f);
  buf[n] = '\0';
  return n > 0;
}

bool read_thread(int tid, ThreadSched* t) {
  char path[64], buf[4096];
  std::snprintf(path, sizeof(path), "/proc/self/task/%d/schedstat", tid);
  if (!read_small(path, buf, sizeof(buf))) return false;
  unsigned long long run = 0, wait = 0;
  if (std::sscanf(buf, "%llu %llu", &run, &wait) != 2) return false;
  t->cpu_ns = run;
  t->delay_ns = wait;
  std::snprintf(path, sizeof(path), "/proc/self/task/%d/status", tid);
  if (read_small(path, buf, sizeof(buf))) {
    if (const char* p = std::strstr(buf, "\nvoluntary_ctxt_switches:")) t->nvcsw = std::strtoull(p + 25, nullptr, 10);
    if (const char* p = std::strstr(buf, "\nnonvoluntary_ctxt_switches:"))
      t->nivcsw = std::strtoull(p + 28, nullptr, 10);
  }
  std::snprintf(path, sizeof(path), "/proc/self/task/%d/stat", tid);
  if (read_small(path, buf, sizeof(buf))) {
    // fields after the parenthesised comm: state is field 3, processor 39
    const char* q = std::strrchr(buf, ')');
    int field = 2;
    for (const char* c = q ? q + 1 : buf; *c; ++c)
      if (*c == ' ' && ++field == 39) {
        t->cpu = std::atoi(c + 1);
        break;
      }
  }
  return true;
}

// /proc/softirqs rows for the given CPUs.
std::map<int, std::map<std::string, uint64_t>> read_softirqs(const std::set<int>& cpus) {
  std::map<int, std::map<std::string, uint64_t>> out;
  if (cpus.empty()) return out;
  FILE* f = std::fopen("/proc/softirqs", "r");
  if (!f) return out;
  std::vector<int> cols;
  char* line = nullptr;
  size_t cap = 0;
  bool header = true;
  while (getline(&line, &cap, f) > 0) {
    if (header) {
      for (char* tok = std::strtok(line, " \t\n"); tok; tok = std::strtok(nullptr, " \t\n"))
        if (std::strncmp(tok, "CPU", 3) == 0) cols.push_back(std::atoi(tok + 3));
      header = false;
      continue;
    }
    char* colon = std::strchr(line, ':');
    if (!colon) continue;
    *colon = '\0';
    std::string kind(line);
    kind.erase(0, kind.find_first_not_of(' '));
    char* p = colon + 1;
    for (size_t i = 0; i < cols.size(); ++i) {
      char* end = nullptr;
      const unsigned long long v = std::strtoull(p, &end, 10);
      if (end == p) break;
      p = end;
      if (cpus.count(cols[i])) out[cols[i]][kind] = v;
    }
  }
  std::free(line);
  std::fclose(f);
  return out;
}

// "<Prefix>: name name ...\n<Prefix>: v v ..." tables (/proc/net/snmp,
// /proc/net/netstat): the wanted fields of the row with this prefix.
void read_proto_table(const char* path, const char* prefix, const std::vector<const char*>& want,
                      std::map<std::string, uint64_t>* out) {
  FILE* f = std::fopen(path, "r");
  if (!f) return;
  char* line = nullptr;
  size_t cap = 0;
  std::vector<std::string> names;
  const size_t plen = std::strlen(prefix);
  while (getline(&line, &cap, f) > 0) {
    if (std::strncmp(line, prefix, plen) != 0) continue;
    std::vector<std::string> toks;
    for (char* tok = std::strtok(line + plen, " \t\n"); tok; tok = std::strtok(nullptr, " \t\n")) toks.emplace_back(tok);
    if (names.empty()) {
      names = std::move(toks);
      continue;
    }
    for (size_t i = 0; i < names.size() && i < toks.size(); ++i)
      for (const char* w : want)
        if (names[i] == w) (*out)[w] = std::strtoull(toks[i].c_str(), nullptr, 10);
    break;
  }
  std::free(line);
  std::fclose(f);
}

// /proc/net/softnet_stat rows (hex): processed, dropped, time_squeeze, ...,
// the CPU id in column 12 on current kernels (the row index otherwise).
std::map<int, std::pair<uint64_t, uint64_t>> read_softnet(const std::set<int>& cpus) {
  std::map<int, std::pair<uint64_t, uint64_t>> out;
  if (cpus.empty()) return out;
  FILE* f = std::fopen("/proc/net/softnet_stat", "r");
  if (!f) return out;
  char* line = nullptr;
  size_t cap = 0;
  int row = 0;
  while (getline(&line, &cap, f) > 0) {
    unsigned long long v[13] = {0};
    int n = 0;
    char* p = line;
    while (n < 13) {
      char* end = nullptr;
      const unsigned long long x = std::strtoull(p, &end, 16);
      if (end == p) break;
      v[n++] = x;
      p = end;
    }
    const int cpu = n > 12 ? static_cast<int>(v[12]) : row;
    if (n >= 3 && cpus.count(cpu)) out[cpu] = {v[1], v[2]};
    ++row;
  }
  std::free(line);
  std::fclose(f);
  return out;
}

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}
}  // namespace

void register_named_thread(const char* name) {
  const int tid = static_cast<int>(::syscall(SYS_gettid));
  std::lock_guard<std::mutex> lk(g_mu);
  registry()[tid] = name;
}

SchedSample sched_sample(const std::vector<std::string>& prefixes) {
  std::vector<std::pair<int, std::string>> want;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    for (const auto& [tid, name] : registry())
      for (const auto& p : prefixes)
        if (name.compare(0, p.size(), p) == 0) {
          want.emplace_back(tid, name);
          break;
        }
  }
  SchedSample s;
  s.t_ns = mono_ns();
  std::set<int> cpus, dead;
  for (const auto& [tid, name] : want) {
    ThreadSched t;
    t.tid = tid;
    t.name = name;
    if (!read_thread(tid, &t)) {
      dead.insert(tid);
      continue;
    }
    if (t.cpu >= 0) cpus.insert(t.cpu);
    s.threads.push_back(std::move(t));
  }
  if (!dead.empty()) {  // exited threads (tids may be reused: forget them)
    std::lock_guard<std::mutex> lk(g_mu);
    for (int tid : dead) registry().erase(tid);
  }
  s.softirqs = read_softirqs(cpus);
  s.softnet = read_softnet(cpus);
  read_proto_table("/proc/net/snmp", "Tcp:", {"RetransSegs"}, &s.tcp);
  read_proto_table("/proc/net/netstat", "TcpExt:",
                   {"TCPLossProbes", "TCPTimeouts", "PruneCalled", "RcvPruned", "TCPRcvQDrop", "TCPBacklogDrop",
                    "TCPFastRetrans", "TCPSlowStartRetrans", "TCPSpuriousRtxHostQueues", "TCPSACKReorder",
                    "TCPDSACKRecv"},
                   &s.tcp);
  return s;
}

namespace {
// One helper thread per process; requests are served one at a time.
struct OffcoreSampler {
  std::mutex mu;
  std::condition_variable cv;
  std::function<void()> job;
  bool busy = false;
  std::vector<int> avoid;
  bool started = false;

  void run() {
    // this thread is not registered: it never samples itself
    std::vector<int> cur;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return static_cast<bool>(job); });
      if (avoid != cur) {
        cur = avoid;
        cpu_set_t set;
        CPU_ZERO(&set);
        if (sched_getaffinity(0, sizeof(set), &set) == 0) {
          cpu_set_t keep = set;
          for (int c : cur)
            if (c >= 0 && c < CPU_SETSIZE) CPU_CLR(c, &keep);
          if (CPU_COUNT(&keep) > 0) sched_setaffinity(0, sizeof(keep), &keep);
        }
      }
      auto f = std::move(job);
      job = nullptr;
      lk.unlock();
      f();
      lk.lock();
      busy = false;
      cv.notify_all();
    }
  }
};

OffcoreSampler& offcore() {
  static auto* s = new OffcoreSampler();  // process lifetime (detached thread)
  return *s;
}
}  // namespace

SchedSample sched_sample_offcore(const std::vector<std::string>& prefixes, const std::vector<int>& avoid) {
  OffcoreSampler& o = offcore();
  SchedSample out;
  std::unique_lock<std::mutex> lk(o.mu);
  if (!o.started) {
    o.started = true;
    std::thread([&o] { o.run(); }).detach();
  }
  o.cv.wait(lk, [&] { return !o.busy; });
  o.busy = true;
  bool done = false;
  o.avoid = avoid;
  o.job = [&] {
    SchedSample x = sched_sample(prefixes);
    std::lock_guard<std::mutex> g(o.mu);
    out = std::move(x);
    done = true;
  };
  o.cv.notify_all();
  o.cv.wait(lk, [&] { return done; });
  return out;
}

ReadSchedDiag sched_delta(const SchedSample& a, const SchedSample& b) {
  ReadSchedDiag d;
  d.wall_ms = (b.t_ns - a.t_ns) / 1e6;
  std::map<int, const ThreadSched*> before;
  for (const auto& t : a.threads) before[t.tid] = &t;
  std::set<int> cpus;
  for (const auto& t : b.threads) {
    auto it = before.find(t.tid);
    if (it == before.end()) continue;
    const ThreadSched& x = *it->second;
    if (t.cpu_ns == x.cpu_ns && t.delay_ns == x.delay_ns) continue;  // did not run
    ReadSchedDiag::Row& r = d.threads[t.name];
    r.cpu_ms += (t.cpu_ns - x.cpu_ns) / 1e6;
    r.delay_ms += (t.delay_ns - x.delay_ns) / 1e6;
    r.nivcsw += t.nivcsw - x.nivcsw;
    r.nvcsw += t.nvcsw - x.nvcsw;
    for (int c : {x.cpu, t.cpu})
      if (c >= 0 && std::find(r.cpus.begin(), r.cpus.end(), c) == r.cpus.end()) r.cpus.push_back(c);
    if (t.cpu >= 0) cpus.insert(t.cpu);
  }
  for (int c : cpus) {
    auto ia = a.softirqs.find(c), ib = b.softirqs.find(c);
    if (ia == a.softirqs.end() || ib == b.softirqs.end()) continue;
    for (const auto& [kind, v] : ib->second) {
      auto k = ia->second.find(kind);
      if (k != ia->second.end() && v > k->second) d.softirqs[kind] += v - k->second;
    }
  }
  for (const auto& [c, v] : b.softnet) {
    auto it = a.softnet.find(c);
    if (it == a.softnet.end()) continue;
    if (v.first > it->second.first) d.softnet_dropped += v.first - it->second.first;
    if (v.second > it->second.second) d.softnet_squeeze += v.second - it->second.second;
  }
  for (const auto& [k, v] : b.tcp) {
    auto it = a.tcp.find(k);
    d.tcp[k] = it != a.tcp.end() && v > it->second ? v - it->second : 0;
  }
  return d;
}

}  // namespace gcsb
