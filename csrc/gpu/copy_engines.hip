// SDMA copy engines of a GPU: probe and warm-up.
//
// Measured (profiles/r3_sdma_engines): the first hipMemcpyAsync that lands on an
// SDMA engine the process has not used yet blocks the CALLING thread for
// ~7 ms while the runtime brings that engine's queue up; the copy itself then
// takes 40 us.  Streams are spread over the engines by the runtime, so with 8
// pool streams the first reads, and the first reads of a new block, kept
// finding a cold engine: a 7 ms hand-off inside a 5.6 ms sliced read (its
// p99 of 12.4 ms), the config-5 uploads' 13.6 ms first upload (round 2).
//
// warm_copy_engines() issues one tiny copy per engine and direction through
// the HSA runtime HIP itself runs on (hsa_amd_memory_async_copy_on_engine),
// at stream-pool construction: every engine a later hipMemcpyAsync can pick
// is brought up once, off the timed path.  copy_engine_probe() reports the
// engines, the per-engine first / second copy times, and whether a
// hipDeviceSynchronize() makes an engine cold again.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "core/util.h"
#include "gpu/engine.h"

namespace gcsb {

namespace {

struct Agents {
  hsa_agent_t gpu{0};
  std::vector<hsa_agent_t> cpus;
  bool ok = false;
};

struct FindCtx {
  uint32_t bdf = 0;
  Agents* out = nullptr;
};

hsa_status_t visit_agent(hsa_agent_t a, void* data) {
  auto* c = static_cast<FindCtx*>(data);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU) {
    c->out->cpus.push_back(a);
  } else if (t == HSA_DEVICE_TYPE_GPU) {
    uint32_t bdf = 0;
    if (hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf) == HSA_STATUS_SUCCESS &&
        (bdf >> 3) == (c->bdf >> 3)) {  // bus + device; any function
      c->out->gpu = a;
      c->out->ok = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}

// The HSA agents of HIP device `dev` (matched by PCI bus/device) and the CPUs.
Agents agents_of(int dev) {
  Agents a;
  int bus = 0, devno = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
      hipDeviceGetAttribute(&devno, hipDeviceAttributePciDeviceId, dev) != hipSuccess)
    return a;
  // HIP initialised the runtime; hsa_init only takes a reference on it
  if (hsa_init() != HSA_STATUS_SUCCESS) return a;
  FindCtx c;
  c.bdf = (static_cast<uint32_t>(bus) << 8) | (static_cast<uint32_t>(devno) << 3);
  c.out = &a;
  hsa_iterate_agents(visit_agent, &c);
  if (a.cpus.empty()) a.ok = false;
  return a;
}

// One copy of `n` bytes on `engine` (bit mask); ms, or -1 on error / timeout.
double timed_copy(void* dst, hsa_agent_t dst_agent, const void* src, hsa_agent_t src_agent, size_t n,
                  uint32_t engine, std::string* err) {
  hsa_signal_t s;
  if (hsa_signal_create(1, 0, nullptr, &s) != HSA_STATUS_SUCCESS) {
    *err = "hsa_signal_create";
    return -1;
  }
  const int64_t t0 = now_ns();
  hsa_status_t st = hsa_amd_memory_async_copy_on_engine(dst, dst_agent, src, src_agent, n, 0, nullptr, s,
                                                        static_cast<hsa_amd_sdma_engine_id_t>(engine), true);
  double ms = -1;
  if (st == HSA_STATUS_SUCCESS) {
    // bounded wait: a copy engine that never completes must not hang the caller
    const hsa_signal_value_t v =
        hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_LT, 1, 5000000000ull, HSA_WAIT_STATE_BLOCKED);
    if (v < 1)
      ms = (now_ns() - t0) / 1e6;
    else
      *err = "timeout";
  } else {
    const char* m = nullptr;
    hsa_status_string(st, &m);
    *err = m ? m : "copy failed";
  }
  hsa_signal_destroy(s);
  return ms;
}

struct Bufs {
  void* host = nullptr;
  void* dev = nullptr;
};

Bufs scratch(int dev) {
  static std::mutex mu;
  static std::vector<std::pair<int, Bufs>> all;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& [d, b] : all)
    if (d == dev) return b;
  Bufs b;
  hip_check(hipSetDevice(dev), "hipSetDevice");
  hip_check(hipHostMalloc(&b.host, 8192, hipHostMallocDefault), "hipHostMalloc(engine warm)");
  hip_check(hipMalloc(&b.dev, 8192), "hipMalloc(engine warm)");
  all.emplace_back(dev, b);
  return b;
}

uint32_t engine_mask(const Agents& a, bool h2d) {
  uint32_t m = 0, p = 0;
  const hsa_agent_t dst = h2d ? a.gpu : a.cpus[0], src = h2d ? a.cpus[0] : a.gpu;
  (void)hsa_amd_memory_copy_engine_status(dst, src, &m);
  (void)hsa_amd_memory_get_preferred_copy_engine(dst, src, &p);
  uint32_t num = 0;
  (void)hsa_agent_get_info(a.gpu, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NUM_SDMA_ENG), &num);
  uint32_t all = num >= 16 ? 0xFFFFu : ((1u << num) - 1u);
  return m | p | all;
}

}  // namespace

int warm_copy_engines(int device) {
  static std::mutex mu;
  static std::set<int> done;
  std::lock_guard<std::mutex> lk(mu);
  if (done.count(device)) return 0;
  done.insert(device);
  Agents a = agents_of(device);
  if (!a.ok) return -1;
  Bufs b = scratch(device);
  int warmed = 0;
  for (bool h2d : {true, false}) {
    const uint32_t mask = engine_mask(a, h2d);
    for (int e = 0; e < 16; ++e) {
      if (!(mask & (1u << e))) continue;
      std::string err;
      double ms = h2d ? timed_copy(b.dev, a.gpu, b.host, a.cpus[0], 4096, 1u << e, &err)
                      : timed_copy(static_cast<uint8_t*>(b.host) + 4096, a.cpus[0], b.dev, a.gpu, 4096, 1u << e, &err);
      if (ms >= 0) ++warmed;
      if (err == "timeout") return warmed;  // a stuck engine: do not wait 5 s on each of the others
    }
  }
  return warmed;
}

std::string copy_engine_probe(int device) {
  Agents a = agents_of(device);
  if (!a.ok) return "{\"error\": \"no HSA agent for the device\"}";
  Bufs b = scratch(device);
  uint32_t num = 0, numx = 0;
  (void)hsa_agent_get_info(a.gpu, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NUM_SDMA_ENG), &num);
  (void)hsa_agent_get_info(a.gpu, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_NUM_SDMA_XGMI_ENG), &numx);
  std::string out = "{\"num_sdma\": " + std::to_string(num) + ", \"num_sdma_xgmi\": " + std::to_string(numx) +
                    ", \"cpu_agents\": " + std::to_string(a.cpus.size());
  for (bool h2d : {true, false}) {
    uint32_t m = 0, p = 0;
    const hsa_agent_t dst = h2d ? a.gpu : a.cpus[0], src = h2d ? a.cpus[0] : a.gpu;
    (void)hsa_amd_memory_copy_engine_status(dst, src, &m);
    (void)hsa_amd_memory_get_preferred_copy_engine(dst, src, &p);
    const char* d = h2d ? "h2d" : "d2h";
    char buf[128];
    std::snprintf(buf, sizeof(buf), ", \"%s_status_mask\": %u, \"%s_preferred_mask\": %u", d, m, d, p);
    out += buf;
    out += std::string(", \"") + d + "\": [";
    const uint32_t mask = engine_mask(a, h2d);
    bool first = true;
    for (int e = 0; e < 16; ++e) {
      if (!(mask & (1u << e))) continue;
      double t[3];
      std::string err;
      for (int k = 0; k < 3; ++k) {
        if (k == 2) (void)hipDeviceSynchronize();  // does a device-wide sync make the engine cold again?
        t[k] = h2d ? timed_copy(b.dev, a.gpu, b.host, a.cpus[0], 4096, 1u << e, &err)
                   : timed_copy(static_cast<uint8_t*>(b.host) + 4096, a.cpus[0], b.dev, a.gpu, 4096, 1u << e, &err);
      }
      std::snprintf(buf, sizeof(buf), "%s{\"engine\": %d, \"first_ms\": %.3f, \"second_ms\": %.3f, \"after_sync_ms\": %.3f",
                    first ? "" : ", ", e, t[0], t[1], t[2]);
      out += buf;
      if (!err.empty()) out += ", \"error\": \"" + err + "\"";
      out += "}";
      first = false;
    }
    out += "]";
  }
  out += "}";
  return out;
}

}  // namespace gcsb
