// GPU data plane: pinned host ring -> side HIP stream hipMemcpyAsync -> HBM,
// with CRC32C verified by the CDNA4 kernels.  [new].
//
// Reference hot loop (reference main.go:133-148): NewReader, io.CopyBuffer into
// io.Discard, stop the timer.  Here the transport recv()s each object byte
// once, straight into a page-locked ring slot; a full slot is handed to the
// GPU (one async H2D copy + the two CRC launches + an event on the sink's own
// non-blocking stream) while the transport keeps filling the next slot.  The
// read's timer stops in finish() once the last slot's event has fired: every
// byte is in HBM and every checksum the server sent has been checked.
//
// Streams (round 2): every sink and upload source of a process draws from ONE
// per-device pool of GCSB_STREAMS (default 8; 0 = a private stream per sink)
// non-blocking streams.  A slot's H2D copy, its CRC launch and its
// completion event go on one pool stream, in order, so no cross-stream event
// wait exists; consecutive slots of a sink use consecutive pool streams, so
// slot i's CRC overlaps slot i+1's copy.  Round 1 gave every sink two streams
// of its own (32 streams with 8 sliced streams x 2 sinks, multiplexed on 4
// hardware queues, where one stream's event wait head-of-line blocks others).
//
// Slot state machine (debuggable with GCSB_DEBUG_RING=1 asserts):
//   FREE -> FILLING (transport writes) -> INFLIGHT (copy+kernels queued)
//        -> harvested (event complete, results folded) -> FREE
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <thread>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "gpu/crc32c_gpu.h"
#include "storage/client.h"
#include "net/buffered.h"
#include "storage/sink.h"

namespace gcsb {

class ConnRing;

enum class Landing {
  kRing,    // HBM ring of the same geometry as the host ring (discard semantics)
  kObject,  // whole object laid out contiguously in HBM (up to 288 GB per GPU)
};

struct GpuSinkConfig {
  int device = 0;
  size_t slot_bytes = 8 << 20;
  int slots = 4;
  bool verify = true;  // run the CRC kernels
  // Ring slots in write-combined pinned memory: the receive copy's stores
  // skip the CPU caches (no read-for-ownership, nothing to write back before
  // the copy engine reads them).  The CPU never reads a read sink's ring.
  // Config-3 list-read (8 readers): p50 0.346-0.379 ms against 0.412-0.519
  // with cached THP rings; the one-stream headline showed no gain
  // (profiles/r3_ring_thp/wc).
  bool ring_wc = false;
  Landing landing = Landing::kObject;
  // Slot hand-off (H2D copy + CRC launch + event) on one per-device
  // submitter thread instead of the transport thread.  A stream's receive is
  // bound by its receiving core, and the hand-off's HIP calls (~3 us per slot
  // on the submitter vs ~170 us on a transport thread under HIP runtime lock
  // contention, profiles/r1_markers) come off it: one stream per 256 MiB
  // read 12.5k -> 14.4k MiB/s with 2 MiB slots (profiles/r2_single_stream).
  // On by default from round 2.
  bool async_submit = true;
  // Wait on slot events by blocking (interrupt) instead of spinning: under the
  // GPU box's CPU quota (16 CPUs) spinning waiters steal cycles from the
  // receiving threads.
  bool blocking_sync = true;
  // > 0: wait for a slot's event by polling it (hipEventQuery) with sleeps of
  // this many microseconds instead of hipEventSynchronize, whose blocking wait
  // still spins inside the runtime before it sleeps: a short end-of-read wait
  // (a 1 MiB read's last copy + CRC, tens of us) is then all spin, on a core
  // the connection's receiving thread may share.  Config-3 list-read
  // (profiles/r3_w48_tail): worker CPU 0.052 -> 0.024 CPU-s/GiB over gRPC,
  // 0.23 -> 0.17 over HTTP, same MiB/s.  0 = the runtime's blocking wait.
  int wait_poll_us = 10;
  // Attribution A/B only (scripts/experiments/recv_cost_ab.py): what reads a
  // filled ring slot.  kH2D is the data plane; kNone hands the slot straight
  // back (nothing reads the ring: the receive copy alone); kHostRead has the
  // submitter thread read it (host CRC32C) instead of the copy engine.  The
  // two A/B stages land nothing in HBM and verify nothing.
  enum class Stage { kH2D, kNone, kHostRead };
  Stage stage = Stage::kH2D;
  // Multiplexed gRPC (one connection's reader thread feeds every worker's
  // sink): receive into this connection-wide ring instead of a ring per sink.
  // 48 per-worker rings of 2 x 2 MiB are 192 MiB of receive destinations, far
  // past the reader's L3, and a one-stream read into a ring that size pays
  // the same 0.056-0.066 CPU-s/GiB as the multiplexed reader
  // (profiles/r4_bigring); one 4 x 1 MiB ring per connection stays L3-hot
  // (profiles/r4_ringgeom).
  // Object landing with CRC verification only; not owned by the sink.
  ConnRing* conn_ring = nullptr;
  // Cached rings live in one contiguous pinned region and a receive window
  // runs on into the next slot when it is free (GpuSink::acquire); false:
  // every window stops at its slot's end (A/B).
  bool ring_span = true;
};

struct GpuSinkStats {
  uint64_t slots_submitted = 0;
  uint64_t segments = 0;
  uint64_t chunks_verified_gpu = 0;   // whole chunk checked by the K2 epilogue
  uint64_t chunks_verified_host = 0;  // chunk spanning slots, folded on host
  uint64_t objects_verified = 0;
  uint64_t slot_waits = 0;            // transport had to wait for a free slot
  double slot_wait_s = 0;
  uint64_t flag_reuses = 0;           // slots reused on the kernel's host-visible status (no HIP call)
  double handoff_s = 0;               // receiving thread inside the slot hand-off (submit + take, waits included)
};

class GpuSink : public Sink {
  friend class ConnRing;

 public:
  explicit GpuSink(const GpuSinkConfig& cfg);
  ~GpuSink() override;
  GpuSink(const GpuSink&) = delete;
  GpuSink& operator=(const GpuSink&) = delete;

  // Land objects in caller-owned HBM (e.g. a torch tensor) instead of the
  // sink's own buffer. cap must cover the object.
  void set_external_destination(void* dptr, size_t cap);
  void* object_device_ptr() const { return obj_dst_; }
  size_t object_capacity() const { return obj_cap_; }
  const GpuSinkStats& stats() const { return stats_; }
  void reset_stats() { stats_ = GpuSinkStats(); }  // between phases (runner warmup -> timed)
  // host ring slots (ptr, bytes): placement diagnostics
  std::vector<std::pair<const void*, size_t>> ring_ranges() const {
    std::vector<std::pair<const void*, size_t>> r;
    for (const Slot& s : slots_) r.emplace_back(s.host, cfg_.slot_bytes);
    return r;
  }
  const GpuSinkConfig& config() const { return cfg_; }

  void begin(const ObjectInfo& info) override;
  void update_info(const ObjectInfo& info) override;
  Window acquire(size_t want) override;
  void commit(size_t n) override;
  void chunk_begin(size_t len) override;
  void chunk_end(bool has_crc, uint32_t crc) override;
  void resume_at(int64_t offset) override;
  SinkResult finish() override;
  void abort() override;

 private:
  struct SegInfo {
    uint64_t slot_off = 0;
    uint64_t obj_off = 0;
    uint32_t len = 0;
    bool closed = false;
    bool chunk_start = false;
    bool chunk_end = false;
    bool has_expected = false;
    bool broken_chunk = false;  // chunk interrupted by a resume
    uint32_t expected = 0;
  };
  struct Slot {
    uint8_t* host = nullptr;
    uint8_t* dev_ring = nullptr;
    size_t used = 0;
    uint64_t obj_off = 0;
    std::vector<SegInfo> segs;
    hipStream_t st = nullptr;     // device pool stream: this slot's copy, CRC launch and event, in order
    int st_idx = -1;              // its index in the pool (-1: private stream)
    hipEvent_t ev = nullptr;      // slot done: copy landed + CRC kernel finished
    uint32_t* tiles = nullptr;    // this slot's CRC tile scratch (slots on different streams run concurrently)
    bool inflight = false;
    // hand-offs posted to the submitter (receiving thread) / issued by it
    // (guarded by sub_mu_): the slot's event is current when they match
    uint64_t posted = 0, issued = 0;
    CrcSegResult* res = nullptr;  // host-mapped, kMaxSeg entries
    CrcSegResult* d_res = nullptr;  // device alias of res
  };
  void enqueue_slot(Slot& s, uint8_t* dst, const CrcBatch* batch);
  void ensure_object_capacity(int64_t size);
  void grow_object_buffer(uint64_t need);
  Slot& take_slot();
  void open_seg(Slot& s);
  void submit_current();
  // conn-ring mode (cfg_.conn_ring)
  Window ring_acquire();
  void ring_commit(size_t n);
  void ring_wait_all();  // this sink's segments submitted and their results collected
  void ring_fold();
  void wait_slot(Slot& s);
  bool done_by_flags(const Slot& s) const;
  void wait_event(hipEvent_t ev);
  void harvest(Slot& s);
  uint32_t shift(uint32_t v, uint64_t nbytes);
  void set_device() const;

  GpuSinkConfig cfg_;
  std::vector<Slot> slots_;
  uint8_t* ring_base_ = nullptr;  // cached rings: all slots in one contiguous pinned region
  bool spill_ = false;           // the last window runs on into the next slot
  int cur_ = -1;         // FILLING slot index or -1
  int next_ = 0;         // next slot to take
  const CrcTables* d_tables_ = nullptr;
  hipStream_t own_stream_ = nullptr;  // GCSB_STREAMS=0: private stream instead of the pool
  uint32_t* d_tiles_ = nullptr;  // slots x tile scratch
  size_t tiles_cap_ = 0;         // tiles per slot scratch
  CrcSegResult* res_host_ = nullptr;
  uint8_t* own_obj_ = nullptr;
  uint8_t* obj_dst_ = nullptr;
  size_t obj_cap_ = 0;
  bool external_dst_ = false;
  // per-read state
  ObjectInfo info_;
  uint64_t delivered_ = 0;
  bool in_chunk_ = false;
  bool chunk_start_pending_ = false;
  bool chunk_broken_ = false;
  uint32_t chunk_raw_ = 0;  // host fold of a multi-slot chunk
  uint64_t chunk_len_ = 0;
  uint32_t obj_raw_ = 0;    // host fold of the whole object
  uint64_t obj_len_ = 0;
  bool mismatch_ = false;
  bool any_checked_ = false;
  std::string detail_;
  // cached x^(8n) operators for the host fold
  uint64_t op_len_[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  uint32_t op_val_[4] = {0, 0, 0, 0};
  int op_rr_ = 0;
  GpuSinkStats stats_;
  uint32_t host_read_sink_ = 0;  // Stage::kHostRead's CRC (keeps the read)
  std::mutex sub_mu_;
  std::condition_variable sub_cv_;
  // conn-ring mode: this read's segments in the shared ring, in delivery
  // (= object) order, and its chunks; ring_res_ / ring_done_ are guarded by
  // the ring's mutex (any thread may collect a slot's results)
  struct RingRes {
    uint64_t obj_off = 0;
    uint32_t len = 0;
    uint32_t raw = 0;
    bool done = false;
    bool failed = false;
  };
  std::vector<RingRes> ring_res_;
  size_t ring_done_ = 0;
  // ring_wait_all sleeps here (with ConnRing::mu_) until a collect makes
  // this sink done, or the poller role is handed to it
  std::condition_variable ring_cv_;
  bool ring_waiting_ = false;
  int ring_open_slot_ = -1;  // ring slot / segment index of this sink's open segment (-1: none)
  size_t ring_open_seg_ = 0;
  uint64_t ring_open_gen_ = 0;  // ... and that slot's fill generation (RSlot::gen)
  // this sink's open segment is the last of the reader's current slot, in
  // the same fill of it, and not submitted yet: more bytes may extend it
  bool ring_extends(const ConnRing& R) const;
  struct ChunkMark {
    uint64_t start = 0, end = 0;
    bool closed = false, has_crc = false, broken = false;
    uint32_t crc = 0;
  };
  std::vector<ChunkMark> chunks_;
};

// One receive ring for every stream of a multiplexed connection (see
// GpuSinkConfig::conn_ring).  The connection's reader thread fills it through
// the sinks' acquire / commit, segment by segment (a segment: consecutive
// bytes of one stream); a slot goes to the device submitter when full, one
// H2D copy per segment to its own object's HBM offset plus one CRC launch for
// all the slot's segments.  A worker finishing its read submits what the
// reader is not writing into (a slot may go in several parts) and collects
// its segments' results as the kernel publishes them (no HIP call).  The
// reader reuses a slot once every segment's result was collected.
class ConnRing {
 public:
  ConnRing(int device, size_t slot_bytes, int slots);
  ~ConnRing();
  ConnRing(const ConnRing&) = delete;
  ConnRing& operator=(const ConnRing&) = delete;
  struct Stats {
    uint64_t slots_filled = 0, submissions = 0, segments = 0, reader_waits = 0;
    double reader_wait_s = 0;
    uint64_t finish_polls = 0;   // status-word polls by the finishing workers' one poller
    uint64_t finish_sleeps = 0;  // finishing workers that slept on their own condition variable
  };
  Stats stats() const;
  int device() const { return device_; }

 private:
  friend class GpuSink;
  struct Seg {
    GpuSink* owner = nullptr;
    size_t seq = 0;       // index in owner->ring_res_
    uint32_t slot_off = 0;
    uint32_t len = 0;
    uint8_t* dst = nullptr;  // HBM: owner's landing + object offset
  };
  struct RSlot {
    uint8_t* host = nullptr;
    size_t used = 0;
    std::vector<Seg> segs;
    size_t submitted = 0;  // segs handed to the submitter
    size_t collected = 0;  // segs whose results were copied out
    bool filling = false;  // the reader's current slot
    // fills of this slot so far: a sink's remembered (slot, segment) from an
    // earlier fill must never extend another sink's segment that now sits at
    // the same index (with 16 KiB frames of 12 streams a slot wraps between
    // two frames of one stream)
    uint64_t gen = 0;
    hipStream_t st = nullptr;
    int st_idx = -1;
    uint32_t* tiles = nullptr;
    CrcSegResult* res = nullptr;
    CrcSegResult* d_res = nullptr;
  };
  // all under mu_
  void submit_locked(int slot, size_t upto);
  void collect_locked(RSlot& s);
  void flush_locked();  // submit every segment the reader is not writing into
  RSlot& take_slot_locked(std::unique_lock<std::mutex>& lk);
  bool owner_done_locked(const GpuSink* g) const { return g->ring_done_ == g->ring_res_.size(); }
  void collect_all_locked();
  // the finishing worker that polls the kernel's status words for every
  // waiting sink (one at a time: 48 pollers on mu_ starved the reader)
  void hand_off_poller_locked();

  int device_;
  // result entries per slot (a sink takes a new slot when they run out)
  size_t res_cap_ = 0;
  bool poller_ = false;
  std::vector<GpuSink*> waiters_;
  size_t slot_bytes_;
  std::vector<RSlot> slots_;
  int cur_ = -1, next_ = 0;
  bool window_open_ = false;  // the reader is receiving into the last segment of cur_
  const GpuSink* window_owner_ = nullptr;  // ... which belongs to this sink
  const CrcTables* d_tables_ = nullptr;
  uint32_t* d_tiles_ = nullptr;
  size_t tiles_cap_ = 0;
  CrcSegResult* res_host_ = nullptr;
  uint64_t posted_ = 0;
  uint64_t issued_ = 0;
  Stats stats_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
};

// Upload source for the write path (config 5): HBM -> pinned ring via
// hipMemcpyAsync D2H on a side stream, `slots` copies kept in flight ahead of
// the transport.  CRC32C on the GPU from HBM, per staged slot: each slot's
// copy is followed on its stream by one CRC launch over the slot's range
// (a segment per chunk of the message grid), results in host-mapped memory,
// so a message's CRC is ready when its slot's event is; the object CRC is the
// host combine of the chunk CRCs, known once every slot was staged.  Round 5
// ran one synchronous whole-object gpu_crc32c in the constructor instead: a
// launch + sync before the first D2H of every upload.
class GpuByteSource : public ByteSource {
 public:
  GpuByteSource(int device, const void* dptr, uint64_t n, size_t slot_bytes, int slots, bool gpu_crc = true,
                bool async_stage = true);
  ~GpuByteSource() override;
  uint64_t size() const override { return n_; }
  std::pair<const uint8_t*, size_t> next(size_t max) override;
  void seek(uint64_t off) override;
  bool has_crc32c() const override { return has_crc_; }
  uint32_t crc32c() const override;
  bool crc32c_ready() const override;
  // Ranges on the chunk grid (start on a grid multiple, end on one or at the
  // object end) are answered from the GPU-computed chunk CRCs.
  bool range_crc32c(uint64_t off, size_t len, uint32_t* crc) override;
  uint64_t copies() const { return copies_.load(std::memory_order_relaxed); }
  uint64_t gpu_range_crcs() const { return range_hits_; }
  // time next() waited for staged bytes (a slot's issue on the submitter,
  // its D2H copy + CRC): the upload's sender stalled on the staging
  int64_t stage_wait_ns() const { return stage_wait_ns_; }
  // Whole-object staging issues its first kSyncSlots slots on the calling
  // thread and hands the rest (a D2H copy, a CRC launch and an event each)
  // to the device's submitter thread, so the upload's first byte does not
  // wait for ~3 HIP calls per slot of the whole object (setup was 0.44 -
  // 0.57 ms of a 3.5 ms 64 MiB upload, profiles/r6_e).
  static constexpr int kSyncSlots = 2;
  // Objects up to kWholeRingMax stage into a
  // ring that holds all of them: no slot is refilled during the upload, so
  // the transport can splice the staged pages instead of copying them.
  // Larger objects (or parts) keep the bounded refilling ring of `slots`
  // slots and are sent by copy: pinned staging per upload stays at most
  // 64 MiB (the config-5 object) whatever the object size, within the
  // pinned pool's 1 GiB.
  bool stable_until_done() const override {
    return static_cast<uint64_t>(nslots_) * slot_bytes_ >= n_;
  }
  static constexpr uint64_t kWholeRingMax = uint64_t(64) << 20;

 private:
  void restart(uint64_t off);
  void issue(int slot, uint64_t off);
  void wait_all();
  void harvest(int slot) const;  // slot's event done: its chunk CRCs into chunk_crc_
  void await_issued(int slot) const;  // slot issued (or the async issue failed: throws)
  void await_async() const;           // the submitter's issue job finished
  // asynchronous staging (kSyncSlots): slots [0, issued_) are issued;
  // async_busy_ while the submitter's job runs (amu_)
  bool async_stage_ = true;
  std::atomic<int> issued_{0};
  mutable std::mutex amu_;
  mutable std::condition_variable acv_;
  bool async_busy_ = false;
  std::string async_err_;
  int device_;
  const uint8_t* src_;
  uint64_t n_;
  size_t slot_bytes_;
  int nslots_;
  std::vector<hipStream_t> st_;  // per slot, from the device stream pool
  std::vector<int> st_idx_;      // their pool indices (slow-call reports)
  hipStream_t own_stream_ = nullptr;
  std::vector<uint8_t*> host_;
  std::vector<hipEvent_t> ev_;
  std::vector<uint64_t> slot_off_;  // object offset held by each slot (~0 = idle)
  std::vector<size_t> slot_len_;
  uint64_t pos_ = 0;        // next byte the consumer gets
  uint64_t next_issue_ = 0; // next object offset to prefetch
  int cur_ = 0;
  bool has_crc_ = false;
  mutable bool crc_done_ = false;
  mutable uint32_t crc_ = 0;
  std::atomic<uint64_t> copies_{0};
  uint64_t grid_ = 0;                // message grid of range_crc32c (0 = none)
  uint64_t chunk_ = 0;               // CRC chunk: grid_, or the slot when there is no grid
  mutable std::vector<uint32_t> chunk_crc_;  // CRC32C of [i*chunk_, min((i+1)*chunk_, n_))
  mutable std::vector<char> chunk_known_;
  mutable size_t chunks_known_ = 0;
  struct SlotCrc {
    uint32_t* tiles = nullptr;  // tile scratch (pooled per device)
    size_t tiles_cap = 0;
    CrcSegResult* res = nullptr;  // host-mapped results, kMaxSeg entries
    CrcSegResult* d_res = nullptr;
  };
  std::vector<SlotCrc> scr_;
  mutable std::vector<char> slot_harvested_;
  const CrcTables* d_tables_ = nullptr;
  uint64_t range_hits_ = 0;
  int64_t stage_wait_ns_ = 0;
};

// Grow-only HBM buffer (e.g. the landing zone a sliced read's slice sinks
// share: each GpuSink is pointed at base + slice offset).
class DeviceBuffer {
 public:
  explicit DeviceBuffer(int device) : device_(device) {}
  ~DeviceBuffer();
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  uint8_t* ensure(size_t n);  // contents are not preserved on growth
  uint8_t* data() const { return p_; }
  size_t capacity() const { return cap_; }

 private:
  int device_;
  uint8_t* p_ = nullptr;
  size_t cap_ = 0;
};

// Device CRC32C of an arbitrary device range.  chunk > 0: the range is cut
// into chunk-byte segments from its start and each segment's CRC32C is
// appended to *chunks (upload messages' ChecksummedData CRCs); chunk 0 picks
// segment sizes for throughput.
uint32_t gpu_crc32c(int device, const void* dptr, size_t n, size_t chunk = 0,
                    std::vector<uint32_t>* chunks = nullptr);
// Kernel throughput probe: K1+K2 over [dptr, dptr+n) in segments of
// seg_bytes (<= kMaxSeg of them), `iters` back-to-back batches, GB/s.
// tile_log2: 0 = automatic (finalize_crc_batch), 12 / 14 forces 4 / 16 KiB tiles.
// probe: latency probe of the kernel bench (CrcBatch::probe; 0 = full kernel).
double gpu_crc32c_throughput(int device, const void* dptr, size_t n, int iters, size_t seg_bytes, uint32_t* crc0,
                             int tile_log2 = 0, uint32_t probe = 0);
// Fill / verify device memory with synthetic object bytes.
void gpu_fill_pattern(int device, void* dptr, uint64_t n, uint64_t rot, uint64_t obj_off);
uint64_t gpu_verify_pattern(int device, const void* dptr, uint64_t n, uint64_t rot, uint64_t obj_off,
                            uint64_t* first_bad);
int gpu_device_count();
// CPU set of the per-device submitter threads (slot H2D copy + CRC launch
// hand-off); empty = inherit.  Also GCSB_SUBMIT_CPUS=<cpulist>.
void set_submitter_cpus(const std::vector<int>& cpus);
// After a hand-off the per-device submitter polls this long for the next
// one before it sleeps (0 = sleep at once): a post to a polling submitter
// costs the receiving thread no futex wake.  Burns the submitter's core
// (placement aux) while it polls.
void set_submitter_spin_us(int us);

// HIP calls on the slot hand-off / staging path that blocked the calling
// thread (an async copy, launch or event record should return in
// microseconds).  Process-wide; the bench reports them per timed block.
struct SlowHipCalls {
  uint64_t calls = 0;        // hand-off HIP calls timed
  uint64_t slow = 0;         // of them >= the threshold (1 ms)
  double slow_ms_total = 0;
  double max_ms = 0;
  std::string max_call;      // e.g. "hipMemcpyAsync(H2D) stream 3"
};
SlowHipCalls slow_hip_calls();
void reset_slow_hip_calls();
// Issue one tiny async copy on every pool stream of `device` and wait for
// it: the first command on a stream binds its hardware queue lazily, so
// doing it at sink / source construction keeps that cost out of the reads.
void warm_device_streams(int device);

// Pinned <-> HBM copy ceiling in the data plane's own pattern: `total` bytes
// in `chunk`-sized hipMemcpyAsync copies between a ring of `slots` pinned
// chunks (PinnedPool: THP + hipHostRegister, as the sinks' rings) and one HBM
// buffer, round-robin over `streams` pool streams, at most `slots` copies in
// flight (a slot is reused once its event fired).  One untimed pass, then
// `iters` timed passes; GB/s = 1e9 B/s over the timed passes.
struct CopyCeiling {
  double gbps = 0;
  double pass_ms_p50 = 0;
};
// SDMA copy engines (gpu/copy_engines.hip): bring every engine of `device`
// up once with a tiny copy per engine and direction (a cold engine costs the
// first hipMemcpyAsync landing on it ~7 ms); returns the engine/direction
// pairs warmed, 0 if already done, -1 if the HSA agent was not found.
int warm_copy_engines(int device);
// JSON: engine count, availability masks, per-engine first / second /
// after-hipDeviceSynchronize copy times per direction.
std::string copy_engine_probe(int device);
CopyCeiling copy_ceiling(int device, bool h2d, size_t total, size_t chunk, int slots, int streams, int iters);

}  // namespace gcsb
