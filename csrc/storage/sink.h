// Where an object's bytes go as they come off the wire.
//
// Reference: the timed loop copies the reader into io.Discard
// (reference main.go:140) and relies on the storage library for CRC32C checks
// (SURVEY.md C21).  Here the destination is pluggable:
//   DiscardSink  — reference-equivalent CPU baseline (optional host CRC32C);
//   GpuSink      — pinned host ring -> hipMemcpyAsync -> HBM, CRC32C verified by
//                  the CDNA4 kernels (csrc/gpu/).
// Transports drive the protocol below; every method runs on the thread that
// owns the object's byte stream (worker thread for HTTP, connection reader
// thread for multiplexed gRPC).
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace gcsb {

struct ObjectInfo {
  int64_t size = -1;          // full object size, -1 if unknown
  int64_t start_offset = 0;   // first byte delivered (range reads / resumes)
  int64_t generation = 0;
  bool has_crc32c = false;    // whole-object CRC32C (x-goog-hash / object_checksums)
  uint32_t crc32c = 0;
  std::string md5;            // raw 16 bytes if known
};

struct SinkResult {
  uint64_t bytes = 0;
  bool verified = false;      // a checksum was checked and matched
  bool crc_mismatch = false;  // a checksum was checked and did NOT match
  uint32_t computed_crc32c = 0;
  std::string detail;
  int64_t landed_ns = 0;      // steady-clock time the last byte was in its final memory
};

struct Window {
  uint8_t* ptr = nullptr;
  size_t cap = 0;
};

class Sink {
 public:
  virtual ~Sink() = default;
  // A new object read starts (called once per read, before any byte).
  virtual void begin(const ObjectInfo& info) = 0;
  // Object metadata learned after begin (gRPC sends it in the first message).
  virtual void update_info(const ObjectInfo& info) = 0;
  // Writable memory for at least 1 byte; cap may be smaller than `want`.
  virtual Window acquire(size_t want) = 0;
  // `n` bytes were written at the start of the last acquired window.
  virtual void commit(size_t n) = 0;
  // gRPC ChecksummedData framing: a chunk of `len` content bytes follows...
  virtual void chunk_begin(size_t len) { (void)len; }
  // ...and ended; its crc32c if the message carried one.
  virtual void chunk_end(bool has_crc, uint32_t crc) { (void)has_crc; (void)crc; }
  // A retry resumes the stream at object offset `offset` (== bytes delivered).
  virtual void resume_at(int64_t offset) { (void)offset; }
  // All bytes delivered: wait for outstanding async work and verify.
  virtual SinkResult finish() = 0;
  // Abandon the current read (error path): drain async work, no verification.
  virtual void abort() {}
  // Deferred sinks: run queued work on the calling thread (the worker waiting
  // for a multiplexed stream; see DiscardSink's deferred mode).
  virtual void drain() {}
  virtual bool deferred() const { return false; }
  // Deferred sinks: enough is queued that the waiting worker should replay
  // it now rather than at the end of the read (the transport's wake-up is a
  // futex call on the connection's one reader thread).
  virtual bool drain_wanted() const { return true; }
};

// Reference-equivalent sink: bytes land in a reusable host buffer and are
// dropped; CRC32C optionally computed on the host (what the Go library does
// on full HTTP reads).
//
// deferred (multiplexed gRPC / HTTP/2): the connection's reader thread feeds
// every stream of the connection, so a host CRC computed inside commit()
// serialises all streams' checksums behind one core's receive copy
// (profiles/r2_grpc_defer).  In deferred mode the bytes land in chunk_bytes
// THP blocks taken from the process-wide LIFO pool (core/hugebuf.h
// huge_take), commit / chunk_begin /
// chunk_end / resume_at only queue an op, and drain() -- called by the read's
// own worker thread while it waits (poked at every message end) and by
// finish() -- replays the ops in order and hands spent blocks back.  LIFO
// reuse keeps the reader's receive copy landing in cache-warm blocks: with a
// private ring per worker, 48 workers' rings (384 MiB) made every copy
// write-allocate from DRAM.  The reader helps drain only when the sink holds
// kMaxBlocks undrained blocks.
class DiscardSink : public Sink {
 public:
  // copy_out > 0: the reference's EFFECTIVE consumer -- every delivered
  // byte is also copied out in copy_out-byte reads into a small buffer, as
  // io.Discard.ReadFrom pulls 8 KiB Reads out of the library's reader
  // (reference main.go:140): grpc-go decodes whole <= 2 MiB
  // messages, the storage reader serves Read()s out of them.  Runs where the
  // CRC runs (the read's worker thread).  Parity-unpinned: a model of the
  // Go library's copies, not a measurement of it.
  DiscardSink(size_t chunk_bytes, bool host_crc, bool deferred = false, size_t copy_out = 0);
  ~DiscardSink() override;
  void begin(const ObjectInfo& info) override;
  void update_info(const ObjectInfo& info) override;
  Window acquire(size_t want) override;
  void commit(size_t n) override;
  void chunk_begin(size_t len) override;
  void chunk_end(bool has_crc, uint32_t crc) override;
  void resume_at(int64_t offset) override;
  SinkResult finish() override;
  void abort() override;
  void drain() override;
  bool deferred() const override { return deferred_; }
  // two blocks undrained: wake the worker; a 1 MiB object's one block waits
  // for the end-of-stream wake-up instead (one futex call per read, not two)
  bool drain_wanted() const override {
    return held_.load(std::memory_order_relaxed) >= wake_blocks().load(std::memory_order_relaxed);
  }
  // A/B: blocks undrained before the reader wakes the worker (default 2;
  // 0 = at every message end, the round-4 behaviour); set from Python while
  // readers run, hence atomic
  static std::atomic<int>& wake_blocks() {
    static std::atomic<int> n{2};
    return n;
  }

 private:
  struct Op {
    enum Kind : uint8_t { kData, kBegin, kEnd, kResume, kRelease } kind;
    bool has_crc = false;
    uint32_t crc = 0;
    uint64_t off = 0, len = 0;
    uint8_t* blk = nullptr;  // kData: the block holding the bytes; kRelease: block to hand back
  };
  static constexpr int kMaxBlocks = 4;
  void apply_data(const uint8_t* p, size_t n);
  void apply_chunk_begin();
  void apply_chunk_end(bool has_crc, uint32_t crc);
  void apply_resume();
  void push(const Op& op);
  void reset_ring();

  size_t copy_out_ = 0;                  // >0: Read() size of the modelled consumer
  uint64_t copy_sink_ = 0;               // keeps the copied-out bytes observable
  uint8_t* buf_ = nullptr;               // non-deferred: the one reusable buffer
  size_t cap_;
  bool host_crc_;
  bool deferred_;
  uint8_t* cur_ = nullptr;               // deferred: block being filled (reader thread)
  size_t cur_used_ = 0;
  std::atomic<int> held_{0};             // deferred: blocks (huge_take) not yet handed back
  std::mutex qmu_;                       // guards ops_
  std::vector<Op> ops_;
  std::mutex cmu_;                       // one replayer at a time, in order
  std::vector<Op> batch_;
  ObjectInfo info_;
  uint64_t bytes_ = 0;
  uint32_t obj_crc_ = 0;     // running standard crc of all delivered bytes
  uint32_t chunk_crc_ = 0;    // crc of the open chunk's bytes, folded into obj_crc_ at its end
  uint64_t chunk_len_ = 0;
  bool in_chunk_ = false;
  void fold_chunk();
  bool chunk_partial_ = false;
  bool mismatch_ = false;
  bool any_checked_ = false;
  std::string detail_;
};

}  // namespace gcsb
