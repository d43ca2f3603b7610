// Sliced (parallel ranged) read of one object.  [new] — SURVEY.md §2.5
// "Ranged split of a single object across workers: optional extension".
//
// The reference reads every object as ONE stream (reference main.go:134-140:
// NewReader + io.CopyBuffer), so a single object is bound by one TCP stream,
// i.e. one receiving core (~9-16 GB/s on the MI355X hosts' loopback).  A
// sliced read stats the object, then fetches `slices` disjoint byte ranges
// concurrently, each on its own connection (own StorageClient, so gRPC slices
// never share an HTTP/2 connection) and its own sink, each slice landing at
// its offset of the destination.  The object CRC32C is the GF(2) combine of
// the slices' CRCs, checked against the object's stored CRC32C: the read is
// verified end to end exactly like a single-stream read.  The timed region is
// unchanged (request -> every byte landed + verified).
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "storage/client.h"
#include "storage/sink.h"

namespace gcsb {

struct SlicedReadConfig {
  int slices = 4;
  uint64_t min_slice_bytes = 8u << 20;  // smaller objects use fewer slices (1 = plain read)
  std::vector<int> cpus;                // pin the slice threads
  bool verify = true;                   // sinks compute CRCs: check the combined object CRC32C
  // 0: each stream reads one fixed 1/slices share of the object.  >0: the
  // object is cut into pieces of this size (2 MiB multiples) that the streams
  // pull from a shared counter (dynamic load balance: a stream on a slow core
  // takes fewer pieces).  Each stream alternates between two sinks, so one
  // piece's last H2D copies overlap the receive of the next.
  uint64_t piece_bytes = 0;
  // >0: taper the piece size toward the end of the object (guided
  // self-scheduling): each piece is min(piece_bytes, remaining / (2 * streams))
  // rounded up to 2 MiB, but at least this.  The last pieces are small, so the
  // streams finish together instead of one stream still receiving a whole
  // piece while the others idle (the `slice_skew_ms` tail).
  uint64_t piece_min_bytes = 0;
};

class SlicedReader {
 public:
  // make_sink(i): the sink slice i reads into (created once, reused).
  // prepare(total): called once per read, before any slice starts.
  // place(i, sink, offset, len): called for each slice before it starts, on
  // the caller's thread (e.g. point a GpuSink at dst + offset).
  using MakeSink = std::function<std::unique_ptr<Sink>(int)>;
  using Prepare = std::function<void(uint64_t total)>;
  using Place = std::function<void(int, Sink&, uint64_t, uint64_t)>;

  SlicedReader(const ClientConfig& client_cfg, SlicedReadConfig cfg, MakeSink make_sink, Prepare prepare,
               Place place);
  ~SlicedReader();
  SlicedReader(const SlicedReader&) = delete;
  SlicedReader& operator=(const SlicedReader&) = delete;

  ReadResult read(const std::string& bucket, const std::string& object, const volatile bool* cancel = nullptr);
  int slices() const { return cfg_.slices; }
  // Load balance of the reads so far: mean over reads of (last slice's
  // host-landed time - first slice's), i.e. how long the fastest slice idled.
  double mean_skew_ms() const { return reads_ ? skew_ms_sum_ / static_cast<double>(reads_) : 0.0; }
  void reset_skew() { skew_ms_sum_ = 0, reads_ = 0; }
  int num_sinks() const { return static_cast<int>(sinks_.size()); }
  Sink& sink(int i) { return *sinks_[i]; }
  StorageClient& client(int i) { return *clients_[i]; }

 private:
  struct Job {
    std::string bucket, object;
    uint64_t off = 0, len = 0;
    int64_t generation = 0;
    const volatile bool* cancel = nullptr;
    bool pending = false, done = false;
    ReadResult rr;
    std::string error;
    bool retryable = false;
  };
  struct Piece {
    uint64_t off = 0, len = 0;
    ReadResult rr;
    std::string error;
    bool retryable = false;
  };
  void thread_main(int i);
  void run_slice(int i);
  void run_pieces(int i);
  void finish_piece(Sink& s, Piece& p);

  SlicedReadConfig cfg_;
  // piece mode, per read: pieces_ and the shared cursor
  std::vector<Piece> pieces_;
  std::atomic<size_t> next_piece_{0};
  std::atomic<bool> piece_abort_{false};
  std::vector<int64_t> stream_done_ns_;
  Prepare prepare_;
  Place place_;
  std::vector<std::unique_ptr<StorageClient>> clients_;
  std::vector<std::unique_ptr<Sink>> sinks_;
  std::vector<Job> jobs_;
  std::vector<std::thread> threads_;  // slices 1..n-1 (slice 0 runs on the caller)
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  bool stop_ = false;
  double skew_ms_sum_ = 0;
  uint64_t reads_ = 0;
};

}  // namespace gcsb

namespace gcsb {

// Parallel composite upload (the gcloud / gsutil "parallel composite upload"
// technique) [new]: the object is cut into `slices` parts that upload
// concurrently, each on its own connection (own StorageClient) as a temporary
// object, then one compose call assembles the destination and the parts are
// deleted.  Each part's CRC32C is sent with it and checked by the server; the
// composed object's CRC32C must equal the GF(2) combine of the parts' CRCs.
struct SlicedWriteConfig {
  int slices = 8;                       // <= 32 (compose limit)
  uint64_t min_slice_bytes = 8u << 20;
  std::vector<int> cpus;
};

class SlicedWriter {
 public:
  // make_source(i, offset, len): the ByteSource for part i (e.g. a
  // GpuByteSource over HBM [dptr + offset, +len)).
  using MakeSource = std::function<std::unique_ptr<ByteSource>(int, uint64_t, uint64_t)>;

  SlicedWriter(const ClientConfig& client_cfg, SlicedWriteConfig cfg);
  ~SlicedWriter();
  SlicedWriter(const SlicedWriter&) = delete;
  SlicedWriter& operator=(const SlicedWriter&) = delete;

  ObjectMeta write(const std::string& bucket, const std::string& object, uint64_t total, const MakeSource& make_source,
                   const WriteOptions& opt);
  int slices() const { return cfg_.slices; }

 private:
  struct Job {
    std::function<void()> fn;
    bool pending = false, done = false;
    std::string error;
    bool retryable = false;
  };
  void thread_main(int i);
  void run_all(int n);

  SlicedWriteConfig cfg_;
  std::vector<std::unique_ptr<StorageClient>> clients_;
  std::vector<Job> jobs_;
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  bool stop_ = false;
  uint64_t seq_ = 0;
};

}  // namespace gcsb
