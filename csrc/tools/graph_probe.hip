// graph_probe: does a hipGraph make the read pipeline's slot hand-off
// cheaper for the submitter thread?
//
// A slot's GPU work is one H2D copy of a pinned 1 MiB ring slot into the
// object in HBM plus one CRC32C slot-kernel launch, and both change their
// parameters every slot: the copy's destination is the object offset, and the
// kernel's segment table moves with it (csrc/gpu/engine.hip submit path).
// Modes, each over `slots` slots, round-robin on 4 streams (as the ring's):
//   stream       hipMemcpyAsync + launch_crc32c_batch (what the engine does)
//   graph        one captured graph per ring slot; per slot an exec update of
//                the memcpy node and of the kernel node, then hipGraphLaunch
//   graph_fixed  the same graphs relaunched unchanged (the floor: a ring-
//                landing sink whose destinations never move)
// Reports the submitting thread's time per slot (the calls alone), the wall
// time of the whole run, and checks every slot's GPU CRC against the host's.
//
//   graph_probe slots=4000 reps=3
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "core/crc32c.h"
#include "gpu/crc32c_gpu.h"

using namespace gcsb;

namespace {

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
    std::exit(2);
  }
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

constexpr size_t kSlot = 1 << 20;
constexpr int kRing = 4;

struct Ctx {
  uint8_t* host = nullptr;        // kRing pinned slots
  uint8_t* obj = nullptr;         // object in HBM
  size_t obj_bytes = 0;
  const CrcTables* tables = nullptr;
  uint32_t* scratch[kRing] = {};
  CrcSegResult* res_h = nullptr;  // host-mapped, one per slot of the run
  CrcSegResult* res_d = nullptr;
  hipStream_t st[kRing] = {};
};

CrcBatch batch_for(const uint8_t* dst) {
  CrcBatch b;
  std::memset(&b, 0, sizeof b);
  b.nseg = 1;
  b.seg[0].addr = dst;
  b.seg[0].len = kSlot;
  finalize_crc_batch(&b);
  return b;
}

}  // namespace

int main(int argc, char** argv) {
  int slots = 4000, reps = 3;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    if (s.rfind("slots=", 0) == 0) slots = std::atoi(s.c_str() + 6);
    if (s.rfind("reps=", 0) == 0) reps = std::atoi(s.c_str() + 5);
  }
  if (slots < kRing) slots = kRing;
  ck(hipSetDevice(0), "hipSetDevice");
  Ctx c;
  c.obj_bytes = size_t(256) << 20;
  ck(hipHostMalloc(reinterpret_cast<void**>(&c.host), kSlot * kRing, hipHostMallocDefault), "hipHostMalloc ring");
  for (size_t i = 0; i < kSlot * kRing; ++i) c.host[i] = static_cast<uint8_t>(i * 131 + (i >> 20) * 7 + 3);
  ck(hipMalloc(reinterpret_cast<void**>(&c.obj), c.obj_bytes), "hipMalloc object");
  c.tables = device_crc_tables(0);
  const CrcBatch probe_b = batch_for(c.obj);
  for (auto& s : c.scratch) s = crc_scratch_alloc(probe_b.total_tiles + 8);
  ck(hipHostMalloc(reinterpret_cast<void**>(&c.res_h), sizeof(CrcSegResult) * slots,
                   hipHostMallocMapped | hipHostMallocCoherent),
     "hipHostMalloc results");
  ck(hipHostGetDevicePointer(reinterpret_cast<void**>(&c.res_d), c.res_h, 0), "hipHostGetDevicePointer");
  for (auto& s : c.st) ck(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  uint32_t want[kRing];
  for (int r = 0; r < kRing; ++r) want[r] = crc32c(c.host + kSlot * r, kSlot);
  const size_t nobj_slots = c.obj_bytes / kSlot;

  // one captured graph per ring slot: copy into object slot r, CRC it
  hipGraphExec_t exec[kRing];
  hipGraphNode_t copy_node[kRing], crc_node[kRing];
  hipKernelNodeParams kp[kRing];
  for (int r = 0; r < kRing; ++r) {
    hipGraph_t g;
    ck(hipStreamBeginCapture(c.st[r], hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    ck(hipMemcpyAsync(c.obj + kSlot * r, c.host + kSlot * r, kSlot, hipMemcpyHostToDevice, c.st[r]), "capture copy");
    launch_crc32c_batch(batch_for(c.obj + kSlot * r), c.tables, c.scratch[r], c.res_d, c.st[r]);
    ck(hipStreamEndCapture(c.st[r], &g), "hipStreamEndCapture");
    size_t n = 0;
    ck(hipGraphGetNodes(g, nullptr, &n), "hipGraphGetNodes");
    std::vector<hipGraphNode_t> nodes(n);
    ck(hipGraphGetNodes(g, nodes.data(), &n), "hipGraphGetNodes");
    copy_node[r] = crc_node[r] = nullptr;
    for (auto nd : nodes) {
      hipGraphNodeType t;
      ck(hipGraphNodeGetType(nd, &t), "hipGraphNodeGetType");
      if (t == hipGraphNodeTypeMemcpy) copy_node[r] = nd;
      if (t == hipGraphNodeTypeKernel) crc_node[r] = nd;
    }
    if (!copy_node[r] || !crc_node[r] || n != 2) {
      std::fprintf(stderr, "captured graph has %zu nodes, expected one memcpy and one kernel\n", n);
      return 2;
    }
    ck(hipGraphKernelNodeGetParams(crc_node[r], &kp[r]), "hipGraphKernelNodeGetParams");
    ck(hipGraphInstantiate(&exec[r], g, nullptr, nullptr, 0), "hipGraphInstantiate");
  }
  ck(hipDeviceSynchronize(), "sync after capture");

  for (int rep = 0; rep < reps; ++rep)
    for (const char* mode : {"stream", "graph", "graph_fixed"}) {
      const std::string m = mode;
      std::memset(c.res_h, 0xFF, sizeof(CrcSegResult) * slots);
      if (m == "graph_fixed")  // back to the captured copies and kernel arguments
        for (int r = 0; r < kRing; ++r) {
          ck(hipGraphExecMemcpyNodeSetParams1D(exec[r], copy_node[r], c.obj + kSlot * r, c.host + kSlot * r, kSlot,
                                               hipMemcpyHostToDevice),
             "reset copy node");
          CrcBatch b0 = batch_for(c.obj + kSlot * r);
          const CrcTables* tb = c.tables;
          uint32_t* sc = c.scratch[r];
          CrcSegResult* rs = c.res_d + r;
          void* args[] = {&b0, &tb, &sc, &rs};
          hipKernelNodeParams p = kp[r];
          p.kernelParams = args;
          ck(hipGraphExecKernelNodeSetParams(exec[r], crc_node[r], &p), "reset kernel node");
        }
      ck(hipDeviceSynchronize(), "sync");
      double call_s = 0;
      const double t0 = now_s();
      for (int i = 0; i < slots; ++i) {
        const int r = i % kRing;
        uint8_t* dst = c.obj + kSlot * (m == "graph_fixed" ? static_cast<size_t>(r) : i % nobj_slots);
        CrcBatch b = batch_for(dst);
        CrcSegResult* res = c.res_d + i;
        const double c0 = now_s();
        if (m == "stream") {
          ck(hipMemcpyAsync(dst, c.host + kSlot * r, kSlot, hipMemcpyHostToDevice, c.st[r]), "hipMemcpyAsync");
          launch_crc32c_batch(b, c.tables, c.scratch[r], res, c.st[r]);
        } else if (m == "graph_fixed") {
          ck(hipGraphLaunch(exec[r], c.st[r]), "hipGraphLaunch");
        } else {
          {
            ck(hipGraphExecMemcpyNodeSetParams1D(exec[r], copy_node[r], dst, c.host + kSlot * r, kSlot,
                                                 hipMemcpyHostToDevice),
               "hipGraphExecMemcpyNodeSetParams1D");
          }
          // the kernel's arguments: (batch, tables, scratch, results)
          const CrcTables* tb = c.tables;
          uint32_t* sc = c.scratch[r];
          void* args[] = {&b, &tb, &sc, &res};
          hipKernelNodeParams p = kp[r];
          p.kernelParams = args;
          ck(hipGraphExecKernelNodeSetParams(exec[r], crc_node[r], &p), "hipGraphExecKernelNodeSetParams");
          ck(hipGraphLaunch(exec[r], c.st[r]), "hipGraphLaunch");
        }
        call_s += now_s() - c0;
      }
      ck(hipDeviceSynchronize(), "sync");
      const double wall = now_s() - t0;
      int bad = 0;
      // graph_fixed: ring slot r's result lands in entry r every time
      const int checked = m == "graph_fixed" ? kRing : slots;
      for (int i = 0; i < checked; ++i)
        if (c.res_h[i].crc != want[i % kRing] || c.res_h[i].status == kCrcStatusPending) ++bad;
      std::printf("{\"rep\":%d,\"mode\":\"%s\",\"slots\":%d,\"call_us_per_slot\":%.2f,\"wall_us_per_slot\":%.2f,"
                  "\"gbps\":%.2f,\"crc_mismatches\":%d}\n",
                  rep, mode, slots, call_s / slots * 1e6, wall / slots * 1e6,
                  static_cast<double>(kSlot) * slots / wall / 1e9, bad);
      std::fflush(stdout);
    }
  return 0;
}
