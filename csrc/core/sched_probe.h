// Per-read stall attribution: what took the
// receiving or the sending core away from one read.
//
// Every named thread of the process (core/affinity.h name_current_thread)
// is registered here with its tid.  A sample reads, for each registered
// thread whose name matches, the scheduler's view (/proc/self/task/<tid>/
// schedstat: on-CPU and run-queue wait time; status: voluntary and
// involuntary context switches; stat: the CPU it last ran on), and
// /proc/softirqs for the CPUs those threads ran on.  The runner takes one
// sample before a read's timer starts and one after it stops
// (RunnerConfig::read_diag), so the cost (tens of microseconds) stays
// outside every read's latency, and keeps the deltas of its slowest reads.
//
// Reference timed region: /root/reference/main.go:133-145.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace gcsb {

// Called by name_current_thread: remembers (tid, name).
void register_named_thread(const char* name);

struct ThreadSched {
  int tid = 0;
  std::string name;
  uint64_t cpu_ns = 0, delay_ns = 0;  // schedstat: on-CPU, waiting on a run queue
  uint64_t nvcsw = 0, nivcsw = 0;     // context switches: voluntary (blocked), involuntary (preempted)
  int cpu = -1;                       // last CPU
};

struct SchedSample {
  int64_t t_ns = 0;
  std::vector<ThreadSched> threads;
  // softirq counts per CPU of interest: {cpu: {"NET_RX": n, "HRTIMER": n, ...}}
  std::map<int, std::map<std::string, uint64_t>> softirqs;
  // TCP counters of the network namespace (/proc/net/snmp Tcp:, /proc/net/
  // netstat TcpExt:): RetransSegs, TCPLossProbes, TCPTimeouts.  Loopback
  // reader and endpoint share the namespace, so a retransmit by either side
  // shows here (per-socket TCP_INFO would only see the client's own).
  std::map<std::string, uint64_t> tcp;
  // /proc/net/softnet_stat of the CPUs of interest: {cpu: {dropped, time_squeeze}}
  std::map<int, std::pair<uint64_t, uint64_t>> softnet;
};

// Threads whose name starts with one of `prefixes`; softirqs of the CPUs
// they last ran on.
SchedSample sched_sample(const std::vector<std::string>& prefixes);

// The same sample, taken by a helper thread kept off `avoid` (the measured
// placement's CPUs): reading ~30 /proc files costs ~0.5 ms of CPU, which on
// the receiving core's SMT sibling slowed the very reads it attributes
// (profiles/r4_main9 diag100).  The caller blocks meanwhile.
SchedSample sched_sample_offcore(const std::vector<std::string>& prefixes, const std::vector<int>& avoid);

// One read's deltas between two samples, per thread name (summed over
// threads of that name): run-queue delay, involuntary switches, CPU time,
// and the softirqs on the CPUs the receiving / sending threads used.
struct ReadSchedDiag {
  struct Row {
    double cpu_ms = 0, delay_ms = 0;
    uint64_t nivcsw = 0, nvcsw = 0;
    std::vector<int> cpus;
  };
  std::map<std::string, Row> threads;                      // by thread name
  std::map<std::string, uint64_t> softirqs;                // on those CPUs, by kind
  std::map<std::string, uint64_t> tcp;                     // namespace TCP counters over the read
  uint64_t softnet_dropped = 0, softnet_squeeze = 0;       // input-backlog drops / NET_RX budget runs on those CPUs
  double wall_ms = 0;
};
ReadSchedDiag sched_delta(const SchedSample& a, const SchedSample& b);

}  // namespace gcsb
