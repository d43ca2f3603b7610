#include "bench/runner.h"

#include "gpu/markers.h"

#include <sys/resource.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <random>
#include <stdexcept>

#include "core/affinity.h"
#include "core/hugebuf.h"
#include "core/util.h"

namespace gcsb {

namespace {
// gRPC and HTTP/2 multiplex every worker's stream on shared connections: the
// host CRC of a discard sink runs on the worker, not the connection's reader
// (DiscardSink deferred mode).
bool defer_host_crc(const ClientConfig& c) {
  return c.protocol == "grpc" || c.protocol == "http2";
}
}  // namespace


const double kOcLatencyBoundsMs[34] = {1,   2,   3,   4,   5,   6,    8,    10,   13,    16,    20,    25,
                                       30,  40,  50,  65,  80,  100,  130,  160,  200,   250,   300,   400,
                                       500, 650, 800, 1000, 2000, 5000, 10000, 20000, 50000, 100000};

int oc_bucket_index(double v) {
  // OpenCensus: bucket i holds bounds[i-1] <= v < bounds[i]
  int i = 0;
  while (i < 34 && v >= kOcLatencyBoundsMs[i]) ++i;
  return i;
}

double percentile_floor(const std::vector<double>& sorted, int pct) {
  if (sorted.empty()) return 0;
  size_t idx = sorted.size() * static_cast<size_t>(pct) / 100;
  if (idx >= sorted.size()) idx = sorted.size() - 1;
  return sorted[idx];
}

size_t LatencySeries::bin(double ms) {
  // bin 0: <= 2^-20 ms; then 1024 bins per octave up to 2^20 ms (17 min)
  constexpr size_t kBins = 40 * 1024 + 2;
  if (!(ms > 0x1p-20)) return 0;
  const double x = (std::log2(ms) + 20.0) * 1024.0;
  return std::min(kBins - 1, static_cast<size_t>(x) + 1);
}

double LatencySeries::bin_value(size_t b) {
  return b == 0 ? 0.0 : std::exp2((static_cast<double>(b - 1) + 0.5) / 1024.0 - 20.0);
}

void LatencySeries::add(double ms) {
  if (n_ == 0 || ms < min_) min_ = ms;
  if (n_ == 0 || ms > max_) max_ = ms;
  ++n_;
  sum_ += ms;
  if (hist_.empty()) {
    if (exact_.size() < kExact) {
      exact_.push_back(ms);
      return;
    }
    // switch to the histogram: bin every sample so far, drop the samples
    hist_.assign(bin(std::exp2(20.0)) + 1, 0);
    for (double x : exact_) ++hist_[bin(x)];
    std::vector<double>().swap(exact_);
  }
  ++hist_[bin(ms)];
}

void LatencySeries::clear() { *this = LatencySeries(); }

double LatencySeries::pct_floor(int pct) const {
  if (n_ == 0) return 0;
  size_t idx = n_ * static_cast<size_t>(pct) / 100;
  if (idx >= n_) idx = n_ - 1;
  if (hist_.empty()) {
    std::vector<double> v = exact_;
    std::nth_element(v.begin(), v.begin() + idx, v.end());
    return v[idx];
  }
  size_t seen = 0;
  for (size_t b = 0; b < hist_.size(); ++b) {
    seen += hist_[b];
    if (seen > idx) return std::min(max_, std::max(min_, bin_value(b)));
  }
  return max_;
}

Runner::Runner(RunnerConfig cfg) : cfg_(std::move(cfg)) {
  reserve_fd_table();
  if (cfg_.workers <= 0) throw StorageError("worker count not valid", false);
  const GpuSinkConfig& g = cfg_.gpu;
  // one connection carries every worker's stream: gRPC with pool size 1, or
  // HTTP/2 media GETs (always one connection)
  const bool one_conn = (cfg_.client.protocol == "grpc" && cfg_.client.grpc_conn_pool_size == 1) ||
                        cfg_.client.protocol == "http2";
  if (cfg_.conn_ring && cfg_.sink == "gpu" && one_conn && cfg_.workers > 1 && cfg_.slices <= 1 && g.verify &&
      g.landing == Landing::kObject && g.stage == GpuSinkConfig::Stage::kH2D)
    conn_ring_ = std::make_unique<ConnRing>(g.device, cfg_.conn_ring_slot_bytes, cfg_.conn_ring_slots);
  client_ = make_client(cfg_.client);
}

Runner::~Runner() {
  stop();
  wait();
  {
    std::lock_guard<std::mutex> lk(ctl_mu_);
    shutdown_ = true;
  }
  run_cv_.notify_all();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
}

namespace {
void add_gpu_stats(GpuSinkStats& t, const GpuSinkStats& g) {
  t.slots_submitted += g.slots_submitted;
  t.segments += g.segments;
  t.chunks_verified_gpu += g.chunks_verified_gpu;
  t.chunks_verified_host += g.chunks_verified_host;
  t.objects_verified += g.objects_verified;
  t.slot_waits += g.slot_waits;
  t.slot_wait_s += g.slot_wait_s;
  t.flag_reuses += g.flag_reuses;
  t.handoff_s += g.handoff_s;
}
}  // namespace


std::string Runner::object_for(int worker, int64_t seq) const {
  if (!cfg_.object_names.empty()) {
    size_t n = cfg_.object_names.size();
    size_t idx = (static_cast<size_t>(worker) + static_cast<size_t>(seq) * static_cast<size_t>(cfg_.workers)) % n;
    return cfg_.object_names[idx];
  }
  return cfg_.object_prefix + std::to_string(cfg_.worker_id_offset + worker) + cfg_.object_suffix;
}

uintptr_t Runner::landing_ptr(int w) const {
  if (w < 0 || w >= static_cast<int>(sinks_.size())) return 0;
  if (landing_[w]) return reinterpret_cast<uintptr_t>(landing_[w]->data());
  if (gpu_sinks_[w]) return reinterpret_cast<uintptr_t>(gpu_sinks_[w]->object_device_ptr());
  return 0;
}

double Runner::ring_thp_fraction(int w) const {
  if (w < 0 || w >= static_cast<int>(gpu_sinks_.size()) || !gpu_sinks_[w]) return -1;
  long long thp = 0, all = 0;
  for (const auto& [p, n] : gpu_sinks_[w]->ring_ranges()) {
    const long long t = thp_bytes_of(p, n);
    if (t < 0) return -1;
    thp += t;
    all += static_cast<long long>(n);
  }
  return all ? static_cast<double>(thp) / static_cast<double>(all) : -1;
}

std::vector<std::vector<long>> Runner::ring_numa(int w) const {
  std::vector<std::vector<long>> out;
  if (w < 0 || w >= static_cast<int>(gpu_sinks_.size()) || !gpu_sinks_[w]) return out;
  for (const auto& [p, n] : gpu_sinks_[w]->ring_ranges()) out.push_back(numa_nodes_of(p, n));
  return out;
}

void Runner::reset_stats() {
  std::lock_guard<std::mutex> lk(mu_);
  acc_ = RunSummary();
  worker_cpu_s_ = 0;
  lat_ms_.clear();
  host_ms_.clear();
  ttfb_ms_.clear();
  slowest_.clear();
  first_ms_.clear();
  steady_ms_.clear();
  pending_.clear();
  t_first_ = t_last_ = 0;
  start_delay_max_ms_ = 0;
  for (auto& s : sliced_)
    if (s) s->reset_skew();
  // the sinks live across phases: their counters restart with the timed reads
  for (GpuSink* g : gpu_sinks_)
    if (g) g->reset_stats();
  if (cfg_.sink == "gpu")
    for (auto& sr : sliced_)
      if (sr)
        for (int i = 0; i < sr->num_sinks(); ++i) static_cast<GpuSink&>(sr->sink(i)).reset_stats();
  for (auto& g : gpu_stats_) g = GpuSinkStats();
}

void Runner::start() {
  stop_flag_ = false;
  running_ = true;
  if (sinks_.empty()) {
    sinks_.resize(cfg_.workers);
    gpu_sinks_.assign(cfg_.workers, nullptr);
    gpu_stats_.assign(cfg_.workers, GpuSinkStats{});
    sliced_.resize(cfg_.workers);
    landing_.resize(cfg_.workers);
  }
  {
    std::lock_guard<std::mutex> lk(ctl_mu_);
    if (busy_ > 0) throw std::logic_error("Runner::start while a run is in progress");
    start_ns_ = now_ns();
    busy_ = cfg_.workers;
    ++gen_;
    if (threads_.empty())
      for (int w = 0; w < cfg_.workers; ++w) threads_.emplace_back([this, w] { worker_loop(w); });
  }
  run_cv_.notify_all();
}

void Runner::wait() {
  std::unique_lock<std::mutex> lk(ctl_mu_);
  done_cv_.wait(lk, [&] { return busy_ == 0; });
  running_ = false;
}

namespace {
double thread_cpu_s() {
  rusage ru{};
  getrusage(RUSAGE_THREAD, &ru);
  return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}
}  // namespace

void Runner::worker_loop(int w) {
  // pin before the sink allocates its pinned ring: NUMA-local first touch
  pin_current_thread(cfg_.client.cpus);
  name_current_thread("gcsb-worker");
  uint64_t seen = 0;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(ctl_mu_);
      run_cv_.wait(lk, [&] { return shutdown_ || gen_ != seen; });
      if (shutdown_) return;
      seen = gen_;
    }
    const double c0 = thread_cpu_s();
    worker_main(w);
    const double c1 = thread_cpu_s();
    {
      std::lock_guard<std::mutex> lk(mu_);
      worker_cpu_s_ += c1 - c0;  // this run's share of the thread's CPU
    }
    std::lock_guard<std::mutex> lk(ctl_mu_);
    if (--busy_ == 0) done_cv_.notify_all();
  }
}

void Runner::stop() { stop_flag_ = true; }

void Runner::record(ReadRecord&& r, double ms, double host_ms) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!recording_.load(std::memory_order_relaxed)) {
    if (!r.ok) {
      ++acc_.errors;
      if (acc_.first_error.empty()) acc_.first_error = "untimed read of object " + r.object + ": " + r.error;
    }
    return;
  }
  ++acc_.reads;
  if (!r.ok) {
    ++acc_.errors;
    if (acc_.first_error.empty()) acc_.first_error = "while reading object " + r.object + ": " + r.error;
  } else {
    acc_.bytes += r.bytes;
    if (r.verified) ++acc_.verified;
    const double ttfb = r.ttfb_ns > r.start_ns ? (r.ttfb_ns - r.start_ns) / 1e6 : 0.0;
    if (slowest_.size() < 3 || ms > slowest_.back().ms) {
      if (slowest_.size() == 3) slowest_.pop_back();
      Slow sl{lat_ms_.size(), ms, host_ms, ttfb, r.diag};
      auto at = std::find_if(slowest_.begin(), slowest_.end(), [&](const Slow& x) { return ms > x.ms; });
      slowest_.insert(at, std::move(sl));
    }
    lat_ms_.add(ms);
    (r.seq == 0 ? first_ms_ : steady_ms_).add(ms);
    host_ms_.add(host_ms);
    if (r.ttfb_ns > r.start_ns) ttfb_ms_.add(ttfb);
    // metric semantics: integer-truncated milliseconds (reference main.go:146)
    acc_.oc_buckets[oc_bucket_index(std::floor(ms))]++;
  }
  acc_.retries += r.attempts > 1 ? static_cast<uint64_t>(r.attempts - 1) : 0;
  if (!t_first_ || r.start_ns < t_first_) t_first_ = r.start_ns;
  if (r.end_ns > t_last_) t_last_ = r.end_ns;
  if (cfg_.keep_records) pending_.push_back(std::move(r));
}

void Runner::worker_main(int w) {
  try {
    if (cfg_.slices > 1 && !sliced_[w]) {
      SlicedReadConfig sc;
      sc.slices = cfg_.slices;
      sc.min_slice_bytes = cfg_.slice_min_bytes;
      sc.piece_bytes = cfg_.slice_piece_bytes;
      sc.piece_min_bytes = cfg_.slice_piece_min_bytes;
      sc.cpus = cfg_.client.cpus;
      const bool gpu = cfg_.sink == "gpu";
      sc.verify = gpu ? cfg_.gpu.verify : cfg_.host_crc;
      DeviceBuffer* land = nullptr;
      if (gpu) {
        landing_[w] = std::make_unique<DeviceBuffer>(cfg_.gpu.device);
        land = landing_[w].get();
      }
      const RunnerConfig& rc = cfg_;
      sliced_[w] = std::make_unique<SlicedReader>(
          cfg_.client, sc,
          [&rc, gpu](int) -> std::unique_ptr<Sink> {
            if (gpu) {
              GpuSinkConfig g = rc.gpu;
              g.landing = Landing::kObject;
              return std::make_unique<GpuSink>(g);
            }
            return std::make_unique<DiscardSink>(rc.client.read_chunk, rc.host_crc, defer_host_crc(rc.client),
                                                 rc.discard_read_bytes);
          },
          [land](uint64_t total) {
            if (land) land->ensure(total);
          },
          [land](int, Sink& sk, uint64_t off, uint64_t) {
            // each slice lands at its offset; the capacity is the rest of
            // the buffer (a ranged read learns the whole object's size)
            if (land) static_cast<GpuSink&>(sk).set_external_destination(land->data() + off, land->capacity() - off);
          });
    }
    if (!sinks_[w] && cfg_.slices <= 1) {
      if (cfg_.sink == "gpu") {
        GpuSinkConfig gc = cfg_.gpu;
        gc.conn_ring = conn_ring_.get();
        auto g = std::make_unique<GpuSink>(gc);
        gpu_sinks_[w] = g.get();
        sinks_[w] = std::move(g);
      } else {
        // multiplexed gRPC: host CRC on the worker thread, not the connection's reader
        sinks_[w] = std::make_unique<DiscardSink>(cfg_.client.read_chunk, cfg_.host_crc, defer_host_crc(cfg_.client),
                                                  cfg_.discard_read_bytes);
      }
    }
  } catch (const std::exception& e) {
    ReadRecord r;
    r.worker = w;
    r.object = object_for(w, 0);
    r.error = std::string("sink setup: ") + e.what();
    r.start_ns = r.end_ns = now_ns();
    record(std::move(r), 0, 0);
    if (cfg_.stop_on_error) stop_flag_ = true;
    return;
  }
  Sink* sink = sinks_[w].get();
  GpuSink* gsink = gpu_sinks_[w];
  SlicedReader* sliced = sliced_[w].get();
  std::mt19937_64 rng(cfg_.seed ? cfg_.seed + static_cast<uint64_t>(w) : std::random_device{}());
  const uint64_t sample_bound = cfg_.trace_sample_rate >= 1.0
                                    ? ~0ull
                                    : static_cast<uint64_t>(cfg_.trace_sample_rate * 9223372036854775808.0);
  const int64_t t_begin = now_ns();
  std::vector<int> diag_avoid = cfg_.diag_avoid_cpus;
  diag_avoid.insert(diag_avoid.end(), cfg_.client.cpus.begin(), cfg_.client.cpus.end());
  {
    int64_t st;
    {
      std::lock_guard<std::mutex> lk(ctl_mu_);
      st = start_ns_;
    }
    const double d = (now_ns() - st) / 1e6;
    std::lock_guard<std::mutex> lk(mu_);
    if (recording_.load(std::memory_order_relaxed)) start_delay_max_ms_ = std::max(start_delay_max_ms_, d);
  }
  for (int64_t i = 0; i < cfg_.reads_per_worker; ++i) {
    if (stop_flag_) break;
    if (cfg_.duration_s > 0 && (now_ns() - t_begin) / 1e9 >= cfg_.duration_s) break;
    ReadRecord r;
    r.worker = cfg_.worker_id_offset + w;
    r.seq = i;
    r.object = object_for(w, i);
    if (cfg_.trace_sample_rate > 0) {
      r.trace_hi = rng();
      r.trace_lo = rng();
      r.span_id = rng() | 1;
      // OTel TraceIDRatioBased: lower 8 bytes of the trace id >> 1 < rate * 2^63
      r.sampled = cfg_.trace_sample_rate >= 1.0 || (r.trace_lo >> 1) < sample_bound;
    }
    // receiving (h2 reader / HTTP worker), sending (endpoint), submitter
    static const std::vector<std::string> kDiagThreads = {"gcsb-h2-reader", "gcsb-srv", "gcsb-worker",
                                                          "gcsb-submit", "gcsb-slice"};
    SchedSample diag0;
    if (cfg_.read_diag) diag0 = sched_sample_offcore(kDiagThreads, diag_avoid);
    RoctxRange rg(sliced ? "gcsb.read_object(sliced)" : "gcsb.read_object");
    r.start_wall_ns = wall_ns();
    r.start_ns = now_ns();
    ReadResult rr;
    bool ok = true;
    try {
      rr = sliced ? sliced->read(cfg_.bucket, r.object, &stop_flag_)
                  : client_->read_object(cfg_.bucket, r.object, *sink, cfg_.range_offset, cfg_.range_limit,
                                         &stop_flag_);
    } catch (const StorageError& e) {
      r.error = std::string("while creating reader object: ") + e.what();
      ok = false;
    } catch (const std::exception& e) {
      r.error = e.what();
      ok = false;
    }
    r.end_ns = now_ns();
    if (cfg_.read_diag)
      r.diag = std::make_shared<ReadSchedDiag>(sched_delta(diag0, sched_sample_offcore(kDiagThreads, diag_avoid)));
    if (!conclude(std::move(r), rr, ok) && cfg_.stop_on_error) {
      stop_flag_ = true;
      break;
    }
  }
  if (gsink) {
    std::lock_guard<std::mutex> lk(mu_);
    gpu_stats_[w] = gsink->stats();
  } else if (sliced && cfg_.sink == "gpu") {
    GpuSinkStats t;
    for (int i = 0; i < sliced->num_sinks(); ++i) add_gpu_stats(t, static_cast<GpuSink&>(sliced->sink(i)).stats());
    std::lock_guard<std::mutex> lk(mu_);
    gpu_stats_[w] = t;
  }
}

bool Runner::conclude(ReadRecord&& r, const ReadResult& rr, bool ok_so_far) {
  if (ok_so_far) {
    r.ttfb_ns = rr.first_byte_ns;
    r.host_done_ns = rr.host_done_ns;
    r.bytes = rr.bytes;
    r.attempts = rr.attempts;
    r.verified = rr.sink.verified;
    r.ok = !rr.sink.crc_mismatch;
    if (!r.ok) r.error = "while reading and discarding content: " + rr.sink.detail;
    if (r.ok && rr.info.size >= 0 && cfg_.range_limit < 0 && cfg_.range_offset == 0 &&
        rr.bytes != static_cast<uint64_t>(rr.info.size)) {
      r.ok = false;
      r.error = "short read: " + std::to_string(rr.bytes) + " of " + std::to_string(rr.info.size) + " bytes";
    }
  }
  const double ms = (r.end_ns - r.start_ns) / 1e6;
  const double host_ms = r.host_done_ns ? (r.host_done_ns - r.start_ns) / 1e6 : ms;
  if (r.ok && cfg_.latency_fd >= 0) {
    char line[64];
    int n = std::snprintf(line, sizeof(line), "%.3fms\n", ms);
    std::lock_guard<std::mutex> lk(out_mu_);
    ssize_t wr = ::write(cfg_.latency_fd, line, static_cast<size_t>(n));
    (void)wr;
  }
  const bool ok = r.ok;
  record(std::move(r), ms, host_ms);
  return ok;
}

std::vector<ReadRecord> Runner::drain() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<ReadRecord> out;
  out.swap(pending_);
  return out;
}

RunSummary Runner::summary(bool percentiles) const {
  std::lock_guard<std::mutex> lk(mu_);
  RunSummary s = acc_;
  s.worker_cpu_s = worker_cpu_s_;
  s.start_delay_max_ms = start_delay_max_ms_;
  s.elapsed_s = t_last_ > t_first_ ? (t_last_ - t_first_) / 1e9 : 0;
  s.mb_per_s = s.elapsed_s > 0 ? s.bytes / 1048576.0 / s.elapsed_s : 0;
  if (!lat_ms_.empty()) s.avg_ms = lat_ms_.sum() / lat_ms_.size();
  if (!percentiles) return s;
  for (const Slow& x : slowest_) {
    s.slowest.push_back({static_cast<double>(x.index), x.ms, x.host_ms, x.ttfb_ms});
    if (x.diag) s.slowest_diag.push_back(*x.diag);
  }
  if (!lat_ms_.empty()) {
    s.avg_ms = lat_ms_.sum() / lat_ms_.size();
    s.p20_ms = lat_ms_.pct_floor(20);
    s.p50_ms = lat_ms_.pct_floor(50);
    s.p90_ms = lat_ms_.pct_floor(90);
    s.p99_ms = lat_ms_.pct_floor(99);
    s.min_ms = lat_ms_.min();
    s.max_ms = lat_ms_.max();
  }
  s.host_p50_ms = host_ms_.pct_floor(50);
  s.host_p99_ms = host_ms_.pct_floor(99);
  if (!ttfb_ms_.empty()) {
    s.ttfb_p50_ms = ttfb_ms_.pct_floor(50);
    s.ttfb_p99_ms = ttfb_ms_.pct_floor(99);
  }
  if (!first_ms_.empty()) {
    s.first_read_p50_ms = first_ms_.pct_floor(50);
    s.first_read_max_ms = first_ms_.max();
  }
  if (!steady_ms_.empty()) {
    s.steady_p50_ms = steady_ms_.pct_floor(50);
    s.steady_p99_ms = steady_ms_.pct_floor(99);
  }
  int nsliced = 0;
  for (const auto& sr : sliced_)
    if (sr) {
      s.slice_skew_ms += sr->mean_skew_ms();
      ++nsliced;
    }
  if (nsliced) s.slice_skew_ms /= nsliced;
  for (const auto& g : gpu_stats_) {
    s.gpu.slots_submitted += g.slots_submitted;
    s.gpu.segments += g.segments;
    s.gpu.chunks_verified_gpu += g.chunks_verified_gpu;
    s.gpu.chunks_verified_host += g.chunks_verified_host;
    s.gpu.objects_verified += g.objects_verified;
    s.gpu.slot_waits += g.slot_waits;
    s.gpu.slot_wait_s += g.slot_wait_s;
    s.gpu.flag_reuses += g.flag_reuses;
    s.gpu.handoff_s += g.handoff_s;
  }
  return s;
}

}  // namespace gcsb
