// CPU placement for the transport threads.
//
// [new] MI355X nodes are 2-socket with 4 GPUs per NUMA node and 8-core L3
// domains (measured on the GPU box: 16 L3 groups, GPUs 0a/23/5a/72 on node 0,
// 8b/a4/d9/f1 on node 1).  Loopback throughput of one object stream swings by
// ~1.5x with scheduler placement, so each rank pins its receive threads (and
// its node-local endpoint's send threads) to cores of its GPU's NUMA node, and
// allocates the pinned ring from that thread (NUMA-local first touch).
#pragma once
#include <string>
#include <vector>

namespace gcsb {

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}
std::vector<int> parse_cpulist(const std::string& s);
// Pins the calling thread to the given CPUs (no-op if empty). Returns success.
bool pin_current_thread(const std::vector<int>& cpus);
// NUMA node of the pages of [p, p+len), sampled every `stride` bytes
// (move_pages query, nothing moves): counts[node] (index kNumaAbsent counts
// pages not present / not queryable).  Diagnostics for host-memory placement.
constexpr int kNumaMaxNodes = 8;
constexpr int kNumaAbsent = kNumaMaxNodes;
std::vector<long> numa_nodes_of(const void* p, size_t len, size_t stride = 1 << 16);
// NUMA node of the CPU this thread runs on now (-1 if unknown).
int current_numa_node();
// Memory policy of this thread: prefer `node` for new pages (-1 = local).
bool prefer_numa_node(int node);
// Memory policy of this thread: new pages only from `node` (-1 = default).
bool bind_numa_node(int node);
// Pages of [p, p+len) (not yet faulted in) only from `node`; false if the
// kernel refused (then placement falls back to first touch).
bool bind_range_to_node(void* p, size_t len, int node);
// Round-robin pick: thread k gets cpus[k % n] (single-CPU pinning) when
// `spread` is set, else the whole set.
std::vector<int> cpus_for(const std::vector<int>& cpus, int k, bool spread);
// Names the calling thread (/proc/<pid>/task/<tid>/comm, 15 chars max) so the
// bench can attribute process CPU time to client / endpoint / GPU threads.
void name_current_thread(const char* name);

}  // namespace gcsb
