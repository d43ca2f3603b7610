// Workload engine: N worker threads, each repeatedly reading one object.
//
// Reference: main() fans out -worker goroutines through an errgroup
// (reference main.go:200-212); each runs ReadObject (main.go:119-156): start a
// span, start the timer, NewReader + io.CopyBuffer(io.Discard), stop the timer,
// record readLatency (integer ms), Close, end the span.  The first error ends
// that worker and fails the run.
//
// Deliberate, documented deviations:
//   Q3  per-worker results instead of a racy shared err;
//   Q4  one "<ms>ms" latency line per read on the latency fd (stdout by
//       default), everything else on stderr;
//   Q11 the first error cancels the other workers (context-cancel semantics);
//   Q12 optional --duration bound next to the reference's read counts.
// Multi-GPU: worker ids are offset by rank*workers so rank r's workers read
// file_<r*W + w> (one reader process per GPU, see parallel/).
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "core/sched_probe.h"
#include "gpu/engine.h"
#include "storage/client.h"
#include "storage/sliced.h"

namespace gcsb {

// OpenCensus ochttp.DefaultLatencyDistribution bounds in ms (reference
// metrics_exporter.go:28 uses it for the read-latency view).
extern const double kOcLatencyBoundsMs[34];
constexpr int kOcBuckets = 35;

struct RunnerConfig {
  ClientConfig client;
  std::string bucket = "princer-working-dirs";          // reference main.go:44
  std::string object_prefix = "princer_100M_files/file_";  // reference main.go:52
  std::string object_suffix;                            // reference main.go:53
  std::vector<std::string> object_names;                // list-read workload: explicit objects
  int workers = 48;                                     // reference main.go:36
  int64_t reads_per_worker = 1000000;                   // reference main.go:38
  double duration_s = 0;                                // 0 = no time bound
  int worker_id_offset = 0;                             // rank * workers
  std::string sink = "discard";                         // discard | gpu
  bool host_crc = true;                                 // discard sink: CRC32C on the host
  // discard sink: >0 models the reference's effective consumer, 8 KiB
  // io.Discard reads copied out of each delivered message (DiscardSink copy_out)
  size_t discard_read_bytes = 0;
  GpuSinkConfig gpu;
  int latency_fd = -1;                                  // write "<ms>ms\n" per read (1 = stdout)
  bool keep_records = true;
  bool stop_on_error = true;
  double trace_sample_rate = 0.0;                       // 0 disables span records
  int64_t range_offset = 0;
  int64_t range_limit = -1;
  // >1: each read is a sliced read (storage/sliced.h): stat, then `slices`
  // concurrent ranged streams on their own connections, one sink each,
  // landing at their offsets of one HBM buffer; object CRC32C combined.
  int slices = 1;
  uint64_t slice_min_bytes = 8u << 20;
  // >0: sliced reads pull pieces of this size from a shared cursor (dynamic
  // load balance across the streams, storage/sliced.h); 0: fixed shares.
  uint64_t slice_piece_bytes = 0;
  uint64_t slice_piece_min_bytes = 0;  // >0: tapered pieces down to this (storage/sliced.h)
  uint64_t seed = 0;
  // Per-read stall attribution (core/sched_probe.h): a scheduler / softirq
  // sample of the receiving, sending, worker and submitter threads before
  // each read's timer starts and after it stops; the slowest reads keep
  // their deltas (RunSummary::slowest_diag).  Off by default: ~tens of us
  // per read, outside the read's latency but inside the run's wall time.
  bool read_diag = false;
  // GPU sink on ONE multiplexed gRPC connection (pool size 1, several
  // workers): every worker's stream lands through one connection ring
  // (GpuSinkConfig::conn_ring) of conn_ring_slots x conn_ring_slot_bytes
  // instead of a ring per worker (profiles/r4_bigring).  4 x 1 MiB, as the
  // one-stream headline: 48 x 100 MiB gRPC -> HBM 19.3k / 21.5k MiB/s against
  // 16.8k / 18.0k with 8 x 1 MiB, 15.4k / 14.1k with 16 x 1 MiB and 13.9k /
  // 15.5k with a ring per worker (profiles/r4_ringgeom).
  bool conn_ring = true;
  size_t conn_ring_slot_bytes = size_t(1) << 20;
  int conn_ring_slots = 4;
  // CPUs the read_diag sampler must not run on (the placement's; the client
  // CPUs are always added): sched_sample_offcore
  std::vector<int> diag_avoid_cpus;
};

struct ReadRecord {
  int32_t worker = 0;
  int64_t seq = 0;
  std::string object;
  int64_t start_wall_ns = 0;
  int64_t start_ns = 0, ttfb_ns = 0, host_done_ns = 0, end_ns = 0;
  uint64_t bytes = 0;
  int32_t attempts = 0;
  bool ok = false, verified = false, sampled = false;
  uint64_t trace_hi = 0, trace_lo = 0, span_id = 0;
  std::string error;
  std::shared_ptr<ReadSchedDiag> diag;  // RunnerConfig::read_diag
};

struct RunSummary {
  uint64_t reads = 0, errors = 0, bytes = 0, retries = 0, verified = 0;
  double elapsed_s = 0;  // first read start -> last read end
  double mb_per_s = 0;   // MiB/s over elapsed
  double avg_ms = 0, p20_ms = 0, p50_ms = 0, p90_ms = 0, p99_ms = 0, min_ms = 0, max_ms = 0;
  double host_p50_ms = 0, host_p99_ms = 0;  // host-landed latency (reference-equivalent stop)
  double ttfb_p50_ms = 0, ttfb_p99_ms = 0;  // request -> first body byte (0 if not recorded)
  // Each worker's first read dials its connection (the reference's lazy
  // http.Client / grpc dial does the same); with few reads per worker those
  // reads are the p99.  Split out so the steady-state tail is visible.
  double first_read_p50_ms = 0, first_read_max_ms = 0, steady_p50_ms = 0, steady_p99_ms = 0;
  double slice_skew_ms = 0;  // sliced reads: mean spread of the slices' host-landed times
  double worker_cpu_s = 0;   // CPU time of the worker threads in the runs since reset_stats (RUSAGE_THREAD)
  // start() -> the first read's start, slowest worker (the workers are
  // parked between runs; a cold hand-off shows here, not in a read)
  double start_delay_max_ms = 0;
  uint64_t oc_buckets[kOcBuckets] = {0};
  // the 3 slowest reads: {index in completion order, ms, host-landed ms, TTFB ms}
  std::vector<std::vector<double>> slowest;
  std::vector<ReadSchedDiag> slowest_diag;  // aligned with slowest (read_diag runs)
  std::string first_error;
  GpuSinkStats gpu;
};

// Floor-index percentile of a sorted vector (reference ssd_test/main.go:158-161).
double percentile_floor(const std::vector<double>& sorted, int pct);
int oc_bucket_index(double ms_truncated);

// One latency series whose memory stays bounded over the reference's default
// run (48 workers x 1,000,000 reads, main.go:36,38): exact samples up to
// kExact, and from there on a log histogram of every sample with 2^-10
// relative bin width (percentiles within 0.04%).  The reference keeps no
// samples at all: OpenCensus folds each into its distribution
// (main.go:146, metrics_exporter.go).
class LatencySeries {
 public:
  static constexpr size_t kExact = size_t(1) << 20;
  void add(double ms);
  void clear();
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  double sum() const { return sum_; }
  double min() const { return min_; }
  double max() const { return max_; }
  // percentile_floor() of the sorted samples while exact; the bin's
  // geometric centre (clamped to [min, max]) after.
  double pct_floor(int pct) const;
  bool exact() const { return hist_.empty(); }

 private:
  static size_t bin(double ms);
  static double bin_value(size_t b);
  std::vector<double> exact_;
  std::vector<uint64_t> hist_;
  size_t n_ = 0;
  double sum_ = 0, min_ = 0, max_ = 0;
};

class Runner {
 public:
  explicit Runner(RunnerConfig cfg);
  ~Runner();
  void start();
  void wait();
  void stop();
  bool running() const { return running_.load(); }
  std::vector<ReadRecord> drain();
  // percentiles=false: counts, bytes, mean and OC buckets only -- O(1) under
  // the lock the workers record into (the CLI's periodic exporter)
  RunSummary summary(bool percentiles = true) const;
  // Per-worker object name (exposed for tests / CLI).
  std::string object_for(int worker, int64_t seq) const;
  // Phased runs (bench warmup -> timed): sinks (pinned ring, HBM landing
  // buffers) and connections survive between start()/wait() cycles.
  void set_reads_per_worker(int64_t n) { cfg_.reads_per_worker = n; }
  // false: the next runs' reads are untimed (a bench arm's re-warm read
  // between chunks): they count nowhere but a failure still counts as an
  // error of the run.  Set between runs only.
  void set_recording(bool on) { recording_ = on; }
  void reset_stats();
  StorageClient& client() { return *client_; }
  // HBM address worker w's last object landed at (GPU sink, object landing;
  // sliced reads: the shared landing buffer), 0 if none.
  uintptr_t landing_ptr(int w) const;
  // the connection ring's counters (nullptr stats when there is none)
  const ConnRing* conn_ring() const { return conn_ring_.get(); }
  // NUMA placement of worker w's pinned ring, per slot (affinity.h numa_nodes_of)
  std::vector<std::vector<long>> ring_numa(int w) const;
  // Fraction of worker w's pinned ring backed by transparent huge pages
  // (-1 unknown): a 4 KiB-page ring makes every receive copy TLB-bound.
  double ring_thp_fraction(int w) const;

 private:
  void worker_loop(int w);
  void worker_main(int w);
  void record(ReadRecord&& r, double ms, double host_ms);
  // r.end_ns stamped by the caller: fill the record from rr, write the
  // latency line, record it; false = the read failed
  bool conclude(ReadRecord&& r, const ReadResult& rr, bool ok_so_far);
  RunnerConfig cfg_;
  // before client_: destroyed after the connections (their reader threads
  // fill it) and after the sinks whose segments it holds
  std::unique_ptr<ConnRing> conn_ring_;
  std::unique_ptr<StorageClient> client_;
  // The workers live as long as the Runner: created by the first start(),
  // parked between runs (a bench's chunks, warm-up -> timed), woken by the
  // next start().  A run ends when every worker finished its reads.
  std::vector<std::thread> threads_;
  std::mutex ctl_mu_;
  std::condition_variable run_cv_, done_cv_;
  uint64_t gen_ = 0;       // runs started (ctl_mu_)
  int busy_ = 0;           // workers still in the current run (ctl_mu_)
  bool shutdown_ = false;  // ctl_mu_
  int64_t start_ns_ = 0;   // the current run's start() (ctl_mu_)
  double start_delay_max_ms_ = 0;  // mu_
  std::atomic<bool> running_{false};
  std::atomic<bool> recording_{true};
  volatile bool stop_flag_ = false;
  mutable std::mutex mu_;
  std::vector<ReadRecord> pending_;
  LatencySeries lat_ms_, host_ms_, ttfb_ms_, first_ms_, steady_ms_;
  // the 3 slowest ok reads so far (kept as they complete: nothing per read)
  struct Slow {
    size_t index;
    double ms, host_ms, ttfb_ms;
    std::shared_ptr<ReadSchedDiag> diag;
  };
  std::vector<Slow> slowest_;
  RunSummary acc_;
  double worker_cpu_s_ = 0;  // guarded by mu_
  int64_t t_first_ = 0, t_last_ = 0;
  std::mutex out_mu_;
  std::vector<GpuSinkStats> gpu_stats_;
  std::vector<std::unique_ptr<Sink>> sinks_;
  std::vector<GpuSink*> gpu_sinks_;
  std::vector<std::unique_ptr<SlicedReader>> sliced_;   // per worker (slices > 1)
  std::vector<std::unique_ptr<DeviceBuffer>> landing_;  // per worker (sliced GPU reads)
};

}  // namespace gcsb
