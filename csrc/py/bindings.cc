#include <typeinfo>
#include <exception>
#include <unistd.h>
#include <pthread.h>
#include <fcntl.h>
#include <execinfo.h>
// Python bindings (_native): the Python layer only orchestrates (CLI flags,
// exporters, torch.distributed barriers); every hot loop runs in this module
// with the GIL released.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "bench/runner.h"
#include "core/affinity.h"
#include "core/ceiling.h"
#include "core/hugebuf.h"
#include "core/content.h"
#include "core/crc32c.h"
#include "core/util.h"
#include "gpu/crc_types.h"
#include "gpu/engine.h"
#include "h2/h2_client.h"
#include "h2/hpack.h"
#include "proto/storage_v2.h"
#include "server/fakegcs.h"
#include "storage/auth.h"
#include "storage/client.h"
#include "storage/sliced.h"

namespace py = pybind11;
using namespace gcsb;

namespace {

template <typename T>
T get_or(const py::dict& d, const char* k, T dflt) {
  if (d.contains(k) && !d[k].is_none()) return d[k].cast<T>();
  return dflt;
}

RetryPolicy retry_from(const py::dict& d) {
  RetryPolicy p;
  std::string mode = get_or<std::string>(d, "retry_mode", "always");
  p.mode = mode == "never" ? RetryMode::kNever : mode == "idempotent" ? RetryMode::kIdempotent : RetryMode::kAlways;
  p.initial_s = get_or<double>(d, "retry_initial_s", 1.0);
  p.max_s = get_or<double>(d, "retry_max_s", 30.0);
  p.multiplier = get_or<double>(d, "retry_multiplier", 2.0);
  p.max_total_s = get_or<double>(d, "retry_max_total_s", 0.0);
  p.max_attempts = get_or<int>(d, "retry_max_attempts", 0);
  return p;
}

ClientConfig client_from(const py::dict& d) {
  ClientConfig c;
  c.protocol = get_or<std::string>(d, "protocol", "http");
  c.endpoint = Endpoint::parse(get_or<std::string>(d, "endpoint", "http://127.0.0.1:8080"));
  c.http_api = get_or<std::string>(d, "http_api", "xml");
  c.user_agent = get_or<std::string>(d, "user_agent", "prince");
  c.max_conns_per_host = get_or<int>(d, "max_conns_per_host", 100);
  c.max_idle_conns_per_host = get_or<int>(d, "max_idle_conns_per_host", 100);
  c.grpc_conn_pool_size = get_or<int>(d, "grpc_conn_pool_size", 1);
  c.read_chunk = get_or<size_t>(d, "read_chunk", 2u << 20);
  c.h2_max_frame_size = get_or<uint32_t>(d, "h2_max_frame_size", c.h2_max_frame_size);
  c.h2_window = get_or<uint32_t>(d, "h2_window", c.h2_window);
  c.h2_span_max_frame = get_or<uint32_t>(d, "h2_span_max_frame", c.h2_span_max_frame);
  if (c.h2_max_frame_size && (c.h2_max_frame_size < 16384 || c.h2_max_frame_size > (1u << 24) - 1))
    throw std::invalid_argument("h2_max_frame_size: 0 (RFC default) or 16384 .. 16777215");
  if (c.h2_window < 65535 || c.h2_window > 0x7FFFFFFFu)
    throw std::invalid_argument("h2_window: 65535 .. 2147483647");
  c.retry = retry_from(d);
  // 0 = kernel TCP autotuning; an explicit size is capped at rmem_max (the
  // bench's one-stream read asks for 64 MiB: profiles/r2_rcvbuf)
  c.sock.rcvbuf = get_or<int>(d, "rcvbuf", 0);
  c.sock.sndbuf = get_or<int>(d, "sndbuf", 0);
  c.sock.io_timeout_ms = get_or<int>(d, "io_timeout_ms", 0);
  c.sock.congestion = get_or<std::string>(d, "tcp_congestion", "");
  c.sock.loopback_rto_min = get_or<bool>(d, "loopback_rto_min", false);
  c.sock.fill_bytes = get_or<size_t>(d, "fill_bytes", c.sock.fill_bytes);
  c.sock.tls_verify = get_or<bool>(d, "tls_verify", true);
  c.sock.tls_ca_file = get_or<std::string>(d, "tls_ca_file", "");
  c.project = get_or<std::string>(d, "project", "gcs-fuse-test");
  if (d.contains("cpus") && !d["cpus"].is_none()) c.cpus = d["cpus"].cast<std::vector<int>>();
  if (d.contains("reader_cpus") && !d["reader_cpus"].is_none())
    c.reader_cpus = d["reader_cpus"].cast<std::vector<int>>();
  std::string auth = get_or<std::string>(d, "auth", "none");
  if (auth == "static") {
    c.token = std::make_shared<StaticTokenSource>(get_or<std::string>(d, "token", ""));
  } else if (auth == "adc" || auth == "key_file") {
    c.token = get_token_source(get_or<std::string>(d, "key_file", ""), kScopeFullControl,
                               get_or<std::string>(d, "token_uri", ""));
  }
  return c;
}

GpuSinkConfig gpu_from(const py::dict& d) {
  GpuSinkConfig g;
  g.device = get_or<int>(d, "device", 0);
  g.slot_bytes = get_or<size_t>(d, "ring_slot_bytes", 8u << 20);
  g.slots = get_or<int>(d, "ring_slots", 4);
  g.verify = get_or<bool>(d, "gpu_verify", true);
  g.landing = get_or<std::string>(d, "landing", "object") == "ring" ? Landing::kRing : Landing::kObject;
  g.async_submit = get_or<bool>(d, "async_submit", g.async_submit);
  g.blocking_sync = get_or<bool>(d, "blocking_sync", g.blocking_sync);
  g.wait_poll_us = get_or<int>(d, "wait_poll_us", g.wait_poll_us);
  g.ring_wc = get_or<bool>(d, "ring_wc", g.ring_wc);
  g.ring_span = get_or<bool>(d, "ring_span", g.ring_span);
  const std::string stage = get_or<std::string>(d, "gpu_stage", "h2d");
  if (stage == "none") g.stage = GpuSinkConfig::Stage::kNone;
  else if (stage == "host_read") g.stage = GpuSinkConfig::Stage::kHostRead;
  else if (stage != "h2d") throw std::invalid_argument("gpu_stage: h2d | none | host_read");
  return g;
}

py::dict sink_result_dict(const ReadResult& rr) {
  py::dict r;
  r["bytes"] = rr.bytes;
  r["attempts"] = rr.attempts;
  r["verified"] = rr.sink.verified;
  r["crc_mismatch"] = rr.sink.crc_mismatch;
  r["computed_crc32c"] = rr.sink.computed_crc32c;
  r["detail"] = rr.sink.detail;
  r["size"] = rr.info.size;
  r["generation"] = rr.info.generation;
  r["has_crc32c"] = rr.info.has_crc32c;
  r["crc32c"] = rr.info.crc32c;
  r["md5"] = py::bytes(rr.info.md5);
  r["first_byte_ns"] = rr.first_byte_ns;
  r["host_done_ns"] = rr.host_done_ns;
  r["landed_ns"] = rr.sink.landed_ns;
  return r;
}

py::dict meta_dict(const ObjectMeta& m) {
  py::dict r;
  r["name"] = m.name;
  r["bucket"] = m.bucket;
  r["size"] = m.size;
  r["generation"] = m.generation;
  r["metageneration"] = m.metageneration;
  r["has_crc32c"] = m.has_crc32c;
  r["crc32c"] = m.crc32c;
  r["md5"] = py::bytes(m.md5);
  r["content_type"] = m.content_type;
  r["updated"] = m.updated;
  return r;
}

// A read's scheduler / softirq deltas (core/sched_probe.h), per thread name.
py::dict sched_diag_dict(const ReadSchedDiag& x) {
  py::dict d, th, si;
  for (const auto& [name, r] : x.threads) {
    py::dict row;
    row["cpu_ms"] = r.cpu_ms;
    row["run_delay_ms"] = r.delay_ms;
    row["nivcsw"] = r.nivcsw;
    row["nvcsw"] = r.nvcsw;
    row["cpus"] = r.cpus;
    th[py::str(name)] = row;
  }
  for (const auto& [k, v] : x.softirqs) si[py::str(k)] = v;
  d["threads"] = th;
  d["softirqs"] = si;
  py::dict tcp;
  for (const auto& [k, v] : x.tcp) tcp[py::str(k)] = v;
  d["tcp"] = tcp;
  py::dict sn;
  sn["dropped"] = x.softnet_dropped;
  sn["time_squeeze"] = x.softnet_squeeze;
  d["softnet"] = sn;
  d["wall_ms"] = x.wall_ms;
  return d;
}

py::dict gpu_stats_dict(const GpuSinkStats& g) {
  py::dict r;
  r["slots_submitted"] = g.slots_submitted;
  r["segments"] = g.segments;
  r["chunks_verified_gpu"] = g.chunks_verified_gpu;
  r["chunks_verified_host"] = g.chunks_verified_host;
  r["objects_verified"] = g.objects_verified;
  r["slot_waits"] = g.slot_waits;
  r["slot_wait_s"] = g.slot_wait_s;
  r["flag_reuses"] = g.flag_reuses;
  r["handoff_s"] = g.handoff_s;
  return r;
}

// Owning wrapper so Python can keep a GPU sink (and its HBM) across reads.
// Parallel composite uploads (storage/sliced.h SlicedWriter) from host bytes
// or from HBM (per-part GpuByteSource: D2H staging ring + GPU CRC32C).
struct PySlicedWriter {
  std::unique_ptr<SlicedWriter> writer;
  explicit PySlicedWriter(const py::dict& d) {
    ClientConfig cc = client_from(d);
    SlicedWriteConfig sc;
    sc.slices = get_or<int>(d, "slices", 8);
    sc.min_slice_bytes = get_or<uint64_t>(d, "slice_min_bytes", 8u << 20);
    sc.cpus = cc.cpus;
    writer = std::make_unique<SlicedWriter>(cc, sc);
  }
  py::dict write_bytes(const std::string& bucket, const std::string& name, const py::bytes& data, bool resumable,
                       size_t chunk_bytes) {
    char* ptr = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(data.ptr(), &ptr, &len) != 0) throw py::error_already_set();
    ObjectMeta m;
    {
      py::gil_scoped_release nogil;
      WriteOptions o;
      o.resumable = resumable;
      o.chunk_bytes = chunk_bytes;
      const auto* base = reinterpret_cast<const uint8_t*>(ptr);
      m = writer->write(bucket, name, static_cast<uint64_t>(len),
                        [base](int, uint64_t off, uint64_t n) -> std::unique_ptr<ByteSource> {
                          return std::make_unique<HostByteSource>(base + off, n);
                        },
                        o);
    }
    return meta_dict(m);
  }
  py::dict write_from_device(const std::string& bucket, const std::string& name, uintptr_t dptr, uint64_t n,
                             int device, bool resumable, size_t chunk_bytes, size_t slot_bytes, int slots,
                             bool async_stage) {
    ObjectMeta m;
    double ms = 0;
    {
      py::gil_scoped_release nogil;
      WriteOptions o;
      o.resumable = resumable;
      o.chunk_bytes = chunk_bytes;
      const auto* base = reinterpret_cast<const uint8_t*>(dptr);
      const int64_t t0 = now_ns();
      m = writer->write(bucket, name, n,
                        [=](int, uint64_t off, uint64_t len) -> std::unique_ptr<ByteSource> {
                          return std::make_unique<GpuByteSource>(device, base + off, len, slot_bytes, slots, true,
                                                                 async_stage);
                        },
                        o);
      ms = (now_ns() - t0) / 1e6;
    }
    py::dict d = meta_dict(m);
    d["upload_ms"] = ms;
    d["parts"] = writer->slices();
    return d;
  }
};

struct PyGpuSink {
  std::unique_ptr<GpuSink> sink;
};

// Sliced reads into caller-owned HBM (e.g. a torch tensor): stat, then N
// concurrent ranged streams, each on its own connection and GpuSink, landing
// at their offsets of [dptr, dptr + cap); object CRC32C combined and checked.
struct PySlicedGpuReader {
  std::unique_ptr<SlicedReader> reader;
  uint8_t* dst = nullptr;
  size_t cap = 0;
  uint64_t need = 0;
  PySlicedGpuReader(const py::dict& d) {
    ClientConfig cc = client_from(d);
    GpuSinkConfig g = gpu_from(d);
    g.landing = Landing::kObject;
    SlicedReadConfig sc;
    sc.slices = get_or<int>(d, "slices", 8);
    sc.min_slice_bytes = get_or<uint64_t>(d, "slice_min_bytes", 8u << 20);
    sc.piece_bytes = get_or<uint64_t>(d, "slice_piece_bytes", 0);
    sc.piece_min_bytes = get_or<uint64_t>(d, "slice_piece_min_bytes", 0);
    sc.cpus = cc.cpus;
    sc.verify = g.verify;
    reader = std::make_unique<SlicedReader>(
        cc, sc, [g](int) -> std::unique_ptr<Sink> { return std::make_unique<GpuSink>(g); },
        [this](uint64_t total) {
          need = total;
          if (total > cap)
            throw StorageError("object (" + std::to_string(total) + " B) larger than the destination (" +
                                   std::to_string(cap) + " B)",
                               false);
        },
        [this](int, Sink& sk, uint64_t off, uint64_t) {
          static_cast<GpuSink&>(sk).set_external_destination(dst + off, cap - off);
        });
  }
  py::dict read_into(const std::string& bucket, const std::string& name, uintptr_t dptr, size_t n) {
    ReadResult rr;
    {
      py::gil_scoped_release nogil;
      dst = reinterpret_cast<uint8_t*>(dptr);
      cap = n;
      rr = reader->read(bucket, name);
    }
    return sink_result_dict(rr);
  }
};

class PyClient {
 public:
  explicit PyClient(const py::dict& cfg) : client_(make_client(client_from(cfg))) {}

  py::dict read(const std::string& bucket, const std::string& name, const std::string& sink_kind, bool host_crc,
                int64_t offset, int64_t limit) {
    ReadResult rr;
    {
      py::gil_scoped_release nogil;
      // "deferred": host CRC replayed by this (waiting) thread, as the runner
      // does for multiplexed gRPC / HTTP/2 reads
      DiscardSink s(client_->config().read_chunk, host_crc, sink_kind == "deferred");
      rr = client_->read_object(bucket, name, s, offset, limit);
    }
    return sink_result_dict(rr);
  }

  py::dict read_gpu(const std::string& bucket, const std::string& name, PyGpuSink& gs, int64_t offset, int64_t limit) {
    ReadResult rr;
    {
      py::gil_scoped_release nogil;
      rr = client_->read_object(bucket, name, *gs.sink, offset, limit);
    }
    py::dict d = sink_result_dict(rr);
    d["device_ptr"] = reinterpret_cast<uintptr_t>(gs.sink->object_device_ptr());
    return d;
  }

  py::bytes read_bytes(const std::string& bucket, const std::string& name, int64_t offset, int64_t limit) {
    // Collecting sink for tests/small objects.
    struct Collect : Sink {
      std::string data;
      size_t used = 0;
      ObjectInfo info;
      void begin(const ObjectInfo& i) override { info = i; data.clear(); used = 0; }
      void update_info(const ObjectInfo&) override {}
      Window acquire(size_t want) override {
        if (data.size() < used + want) data.resize(used + want);
        return Window{reinterpret_cast<uint8_t*>(&data[used]), want};
      }
      void commit(size_t n) override { used += n; }
      SinkResult finish() override {
        data.resize(used);
        SinkResult r;
        r.bytes = used;
        return r;
      }
    } c;
    {
      py::gil_scoped_release nogil;
      client_->read_object(bucket, name, c, offset, limit);
    }
    return py::bytes(c.data);
  }

  py::dict stat(const std::string& bucket, const std::string& name) {
    ObjectMeta m;
    {
      py::gil_scoped_release nogil;
      m = client_->stat_object(bucket, name);
    }
    return meta_dict(m);
  }

  py::dict list(const std::string& bucket, const std::string& prefix, int page_size, const std::string& token,
                const std::string& delimiter) {
    ListResult r;
    {
      py::gil_scoped_release nogil;
      r = client_->list_objects(bucket, prefix, page_size, token, delimiter);
    }
    py::dict d;
    py::list objs;
    for (auto& o : r.objects) objs.append(meta_dict(o));
    d["objects"] = objs;
    d["prefixes"] = r.prefixes;
    d["next_page_token"] = r.next_page_token;
    return d;
  }

  py::list list_all(const std::string& bucket, const std::string& prefix, int page_size) {
    std::vector<ObjectMeta> all;
    {
      py::gil_scoped_release nogil;
      all = client_->list_all(bucket, prefix, page_size);
    }
    py::list out;
    for (auto& o : all) out.append(meta_dict(o));
    return out;
  }

  py::dict write_bytes(const std::string& bucket, const std::string& name, const py::bytes& data, bool resumable,
                       size_t chunk_bytes) {
    // bytes are immutable and `data` holds a reference: upload straight from
    // the Python buffer, without a copy
    char* ptr = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(data.ptr(), &ptr, &len) != 0) throw py::error_already_set();
    ObjectMeta m;
    {
      py::gil_scoped_release nogil;
      HostByteSource src(reinterpret_cast<const uint8_t*>(ptr), static_cast<size_t>(len));
      WriteOptions o;
      o.resumable = resumable;
      o.chunk_bytes = chunk_bytes;
      m = client_->write_object(bucket, name, src, o);
    }
    return meta_dict(m);
  }

  // Write path (config 5): object bytes in HBM -> pinned ring (D2H) -> upload.
  py::dict write_from_device(const std::string& bucket, const std::string& name, uintptr_t dptr, uint64_t n,
                             int device, bool resumable, size_t chunk_bytes, size_t slot_bytes, int slots,
                             bool async_stage) {
    ObjectMeta m;
    double crc_ms = 0, upload_ms = 0;
    uint64_t copies = 0, range_crcs = 0;
    uint32_t crc = 0;
    bool whole = false;
    double done_ms = 0, stage_wait_ms = 0;
    {
      py::gil_scoped_release nogil;
      int64_t t0 = now_ns();
      auto src = std::make_unique<GpuByteSource>(device, reinterpret_cast<const void*>(dptr), n, slot_bytes, slots,
                                                 true, async_stage);
      int64_t t1 = now_ns();
      WriteOptions o;
      o.resumable = resumable;
      o.chunk_bytes = chunk_bytes;
      m = client_->write_object(bucket, name, *src, o);
      int64_t t2 = now_ns();
      crc_ms = (t1 - t0) / 1e6;
      upload_ms = (t2 - t1) / 1e6;
      copies = src->copies();
      range_crcs = src->gpu_range_crcs();
      crc = src->crc32c();
      whole = src->stable_until_done();
      stage_wait_ms = src->stage_wait_ns() / 1e6;
      src.reset();  // staging drained and returned to the pool
      done_ms = (now_ns() - t0) / 1e6;
    }
    py::dict d = meta_dict(m);
    const UploadPhases ph = client_->last_upload();
    py::dict p;
    p["start_rpc_ms"] = ph.start_rpc_ns / 1e6;
    p["first_send_ms"] = ph.first_send_ns / 1e6;
    p["last_send_ms"] = ph.last_send_ns / 1e6;
    p["response_ms"] = ph.response_ns / 1e6;
    // around write_object: the source's setup before it (D2H staging
    // started, buffers taken) and the whole call including the source's
    // teardown after the response
    p["setup_ms"] = crc_ms;
    p["done_ms"] = done_ms;
    p["stage_wait_ms"] = stage_wait_ms;  // the sender waiting for staged bytes
    d["phases"] = p;
    d["gpu_crc32c"] = crc;
    d["staged_whole"] = whole;  // the whole object staged at once (zero-copy sends)
    d["gpu_message_crcs"] = range_crcs;  // upload messages whose CRC came from the GPU
    d["gpu_crc_ms"] = crc_ms;
    d["upload_ms"] = upload_ms;
    d["d2h_copies"] = copies;
    return d;
  }

  py::dict compose(const std::string& bucket, const std::string& dest, const std::vector<std::string>& sources,
                   const std::string& content_type) {
    ObjectMeta m;
    {
      py::gil_scoped_release nogil;
      m = client_->compose_object(bucket, dest, sources, content_type);
    }
    return meta_dict(m);
  }
  void remove(const std::string& bucket, const std::string& name) {
    py::gil_scoped_release nogil;
    client_->delete_object(bucket, name);
  }

  py::dict stats() {
    auto& s = client_->stats();
    py::dict d;
    d["requests"] = s.requests.load();
    d["retries"] = s.retries.load();
    d["bytes_in"] = s.bytes_in.load();
    d["bytes_out"] = s.bytes_out.load();
    d["path"] = client_->transport_path();
    d["transport"] = client_->transport_name();
    d["dials"] = client_->stats().dials.load();
    return d;
  }
  StorageClient& client() { return *client_; }

 private:
  std::unique_ptr<StorageClient> client_;
};

class PyRunner {
 public:
  explicit PyRunner(const py::dict& d) {
    RunnerConfig c;
    c.client = client_from(d);
    c.bucket = get_or<std::string>(d, "bucket", c.bucket);
    c.object_prefix = get_or<std::string>(d, "object_prefix", c.object_prefix);
    c.object_suffix = get_or<std::string>(d, "object_suffix", c.object_suffix);
    if (d.contains("object_names") && !d["object_names"].is_none())
      c.object_names = d["object_names"].cast<std::vector<std::string>>();
    c.workers = get_or<int>(d, "workers", c.workers);
    c.reads_per_worker = get_or<int64_t>(d, "reads_per_worker", c.reads_per_worker);
    c.duration_s = get_or<double>(d, "duration_s", 0.0);
    c.worker_id_offset = get_or<int>(d, "worker_id_offset", 0);
    c.sink = get_or<std::string>(d, "sink", "discard");
    c.host_crc = get_or<bool>(d, "host_crc", true);
    c.discard_read_bytes = get_or<size_t>(d, "discard_read_bytes", 0);
    c.gpu = gpu_from(d);
    c.latency_fd = get_or<int>(d, "latency_fd", -1);
    c.keep_records = get_or<bool>(d, "keep_records", true);
    c.read_diag = get_or<bool>(d, "read_diag", false);
    c.conn_ring = get_or<bool>(d, "conn_ring", c.conn_ring);
    c.conn_ring_slot_bytes = get_or<size_t>(d, "conn_ring_slot_bytes", c.conn_ring_slot_bytes);
    c.conn_ring_slots = get_or<int>(d, "conn_ring_slots", c.conn_ring_slots);
    if (d.contains("diag_avoid_cpus") && !d["diag_avoid_cpus"].is_none())
      c.diag_avoid_cpus = d["diag_avoid_cpus"].cast<std::vector<int>>();
    c.stop_on_error = get_or<bool>(d, "stop_on_error", true);
    c.trace_sample_rate = get_or<double>(d, "trace_sample_rate", 0.0);
    c.range_offset = get_or<int64_t>(d, "range_offset", 0);
    c.range_limit = get_or<int64_t>(d, "range_limit", -1);
    c.slices = get_or<int>(d, "slices", 1);
    c.slice_min_bytes = get_or<uint64_t>(d, "slice_min_bytes", 8u << 20);
    c.slice_piece_bytes = get_or<uint64_t>(d, "slice_piece_bytes", 0);
    c.slice_piece_min_bytes = get_or<uint64_t>(d, "slice_piece_min_bytes", 0);
    c.seed = get_or<uint64_t>(d, "seed", 0);
    runner_ = std::make_unique<Runner>(std::move(c));
  }
  void start() { runner_->start(); }
  void wait() {
    py::gil_scoped_release nogil;
    runner_->wait();
  }
  void stop() { runner_->stop(); }
  py::list drain() {
    std::vector<ReadRecord> recs = runner_->drain();
    py::list out;
    for (auto& r : recs) {
      py::dict d;
      d["worker"] = r.worker;
      d["seq"] = r.seq;
      d["object"] = r.object;
      d["start_wall_ns"] = r.start_wall_ns;
      d["start_ns"] = r.start_ns;
      d["ttfb_ns"] = r.ttfb_ns;
      d["host_done_ns"] = r.host_done_ns;
      d["end_ns"] = r.end_ns;
      d["bytes"] = r.bytes;
      d["attempts"] = r.attempts;
      d["ok"] = r.ok;
      d["verified"] = r.verified;
      d["sampled"] = r.sampled;
      d["trace_hi"] = r.trace_hi;
      d["trace_lo"] = r.trace_lo;
      d["span_id"] = r.span_id;
      d["error"] = r.error;
      out.append(d);
    }
    return out;
  }
  py::dict summary(bool percentiles) {
    RunSummary s = runner_->summary(percentiles);
    py::dict d;
    d["reads"] = s.reads;
    d["errors"] = s.errors;
    d["bytes"] = s.bytes;
    d["retries"] = s.retries;
    d["verified"] = s.verified;
    d["elapsed_s"] = s.elapsed_s;
    d["mib_per_s"] = s.mb_per_s;
    d["avg_ms"] = s.avg_ms;
    d["p20_ms"] = s.p20_ms;
    d["p50_ms"] = s.p50_ms;
    d["p90_ms"] = s.p90_ms;
    d["p99_ms"] = s.p99_ms;
    d["min_ms"] = s.min_ms;
    d["max_ms"] = s.max_ms;
    d["host_p50_ms"] = s.host_p50_ms;
    d["host_p99_ms"] = s.host_p99_ms;
    d["ttfb_p50_ms"] = s.ttfb_p50_ms;
    d["ttfb_p99_ms"] = s.ttfb_p99_ms;
    d["first_read_p50_ms"] = s.first_read_p50_ms;
    d["first_read_max_ms"] = s.first_read_max_ms;
    d["steady_p50_ms"] = s.steady_p50_ms;
    d["steady_p99_ms"] = s.steady_p99_ms;
    d["slice_skew_ms"] = s.slice_skew_ms;
    d["slowest"] = s.slowest;
    py::list sd;
    for (const ReadSchedDiag& x : s.slowest_diag) sd.append(sched_diag_dict(x));
    d["slowest_diag"] = sd;
    d["worker_cpu_s"] = s.worker_cpu_s;
    d["start_delay_max_ms"] = s.start_delay_max_ms;
    py::list b;
    for (int i = 0; i < kOcBuckets; ++i) b.append(s.oc_buckets[i]);
    d["oc_buckets"] = b;
    d["first_error"] = s.first_error;
    d["gpu"] = gpu_stats_dict(s.gpu);
    return d;
  }
  std::string object_for(int w, int64_t seq) { return runner_->object_for(w, seq); }
  uintptr_t landing_ptr(int w) { return runner_->landing_ptr(w); }
  std::vector<std::vector<long>> ring_numa(int w) { return runner_->ring_numa(w); }
  double ring_thp_fraction(int w) { return runner_->ring_thp_fraction(w); }
  py::object conn_ring_stats() {
    const ConnRing* r = runner_->conn_ring();
    if (!r) return py::none();
    const ConnRing::Stats s = r->stats();
    py::dict d;
    d["slots_filled"] = s.slots_filled;
    d["submissions"] = s.submissions;
    d["segments"] = s.segments;
    d["reader_waits"] = s.reader_waits;
    d["reader_wait_s"] = s.reader_wait_s;
    d["finish_polls"] = s.finish_polls;
    d["finish_sleeps"] = s.finish_sleeps;
    return d;
  }
  std::string transport_path() { return runner_->client().transport_path(); }
  void set_reads_per_worker(int64_t n) { runner_->set_reads_per_worker(n); }
  void set_recording(bool on) { runner_->set_recording(on); }
  void reset_stats() { runner_->reset_stats(); }

 private:
  std::unique_ptr<Runner> runner_;
};

class PyServer {
 public:
  explicit PyServer(const py::dict& d) {
    ServerConfig c;
    c.host = get_or<std::string>(d, "host", "127.0.0.1");
    c.port = get_or<int>(d, "port", 0);
    c.require_auth = get_or<bool>(d, "require_auth", false);
    c.jwt_public_key_pem = get_or<std::string>(d, "jwt_public_key_pem", "");
    c.grpc_chunk = get_or<uint64_t>(d, "grpc_chunk", 2u << 20);
    c.sndbuf = get_or<int>(d, "sndbuf", 0);
    c.zero_copy = get_or<bool>(d, "zero_copy", true);
    c.send_vmsplice = get_or<std::string>(d, "send_source", "vmsplice") != "sendfile";
    c.h2_quantum = get_or<size_t>(d, "h2_quantum", c.h2_quantum);
    c.tls_cert_file = get_or<std::string>(d, "tls_cert_file", "");
    c.tls_key_file = get_or<std::string>(d, "tls_key_file", "");
    if (d.contains("cpus") && !d["cpus"].is_none()) c.cpus = d["cpus"].cast<std::vector<int>>();
    if (d.contains("send_cpus") && !d["send_cpus"].is_none()) c.send_cpus = d["send_cpus"].cast<std::vector<int>>();
    if (d.contains("crc_cpus") && !d["crc_cpus"].is_none()) c.crc_cpus = d["crc_cpus"].cast<std::vector<int>>();
    store_ = std::make_shared<ObjectStore>(get_or<bool>(d, "md5", true));
    store_->set_retain_uploads(get_or<bool>(d, "retain_uploads", true));
    c.write_verify = get_or<bool>(d, "write_verify", true);
    srv_ = std::make_unique<FakeGcsServer>(c, store_);
  }
  void start() { srv_->start(); }
  void stop() {
    py::gil_scoped_release nogil;
    srv_->stop();
  }
  int port() const { return srv_->port(); }
  std::string url() const { return srv_->url(); }
  void add_synthetic(const std::string& bucket, const std::string& prefix, const std::string& suffix, int first,
                     int count, uint64_t size) {
    py::gil_scoped_release nogil;
    store_->add_synthetic_range(bucket, prefix, suffix, first, count, size);
  }
  py::dict add_object(const std::string& bucket, const std::string& name, const py::bytes& data) {
    std::string s = data;
    Blob b;
    b.append(s.data(), s.size());
    auto o = store_->put(bucket, name, std::move(b), "");
    py::dict d;
    d["size"] = o->size;
    d["crc32c"] = o->crc32c;
    d["generation"] = o->generation;
    return d;
  }
  py::object object_info(const std::string& bucket, const std::string& name) {
    auto o = store_->get(bucket, name);
    if (!o) return py::none();
    py::dict d;
    d["size"] = o->size;
    d["crc32c"] = o->crc32c;
    d["md5"] = py::bytes(o->md5());
    d["generation"] = o->generation;
    d["synthetic"] = o->synthetic;
    d["rotation"] = o->rot;
    return d;
  }
  py::bytes object_bytes(const std::string& bucket, const std::string& name, uint64_t off, uint64_t n) {
    auto o = store_->get(bucket, name);
    if (!o) throw std::runtime_error("no such object");
    if (off > o->size) off = o->size;
    if (off + n > o->size) n = o->size - off;
    std::string out;
    out.resize(n);
    uint64_t done = 0;
    while (done < n) {
      uint64_t k = std::min<uint64_t>(n - done, 8 << 20);
      std::memcpy(&out[done], o->bytes(off + done, k), k);
      done += k;
    }
    return py::bytes(out);
  }
  void set_faults(const py::dict& d) {
    auto& f = srv_->faults();
    if (d.contains("fail_next")) f.fail_next = d["fail_next"].cast<int>();
    if (d.contains("fail_status")) f.fail_status = d["fail_status"].cast<int>();
    if (d.contains("disconnect_at")) f.disconnect_at = d["disconnect_at"].cast<int64_t>();
    if (d.contains("disconnect_count")) f.disconnect_count = d["disconnect_count"].cast<int>();
    if (d.contains("corrupt_at")) f.corrupt_at = d["corrupt_at"].cast<int64_t>();
    if (d.contains("corrupt_count")) f.corrupt_count = d["corrupt_count"].cast<int>();
    if (d.contains("throttle_bps")) f.throttle_bps = d["throttle_bps"].cast<int64_t>();
    if (d.contains("latency_ms")) f.latency_ms = d["latency_ms"].cast<int>();
    if (d.contains("finalize_delay_ms")) f.finalize_delay_ms = d["finalize_delay_ms"].cast<int>();
    if (d.contains("drop_trailers_count")) f.drop_trailers_count = d["drop_trailers_count"].cast<int>();
    if (d.contains("stall_at")) f.stall_at = d["stall_at"].cast<int64_t>();
    if (d.contains("stall_ms")) f.stall_ms = d["stall_ms"].cast<int>();
    if (d.contains("stall_count")) f.stall_count = d["stall_count"].cast<int>();
  }
  py::dict stats() {
    auto& s = srv_->stats();
    py::dict d;
    d["connections"] = s.connections.load();
    d["http_requests"] = s.http_requests.load();
    d["grpc_calls"] = s.grpc_calls.load();
    d["bytes_sent"] = s.bytes_sent.load();
    d["bytes_received"] = s.bytes_received.load();
    d["faults_injected"] = s.faults_injected.load();
    d["write_recvs"] = s.write_recvs.load();
    d["write_recv_bytes"] = s.write_recv_bytes.load();
    d["auth_failures"] = s.auth_failures.load();
    d["body_sends"] = s.body_sends.load();
    d["body_wall_us"] = s.body_wall_us.load();
    d["tcp_busy_us"] = s.tcp_busy_us.load();
    d["tcp_rwnd_limited_us"] = s.tcp_rwnd_limited_us.load();
    d["tcp_sndbuf_limited_us"] = s.tcp_sndbuf_limited_us.load();
    d["tcp_cwnd_bytes_sum"] = s.tcp_cwnd_bytes_sum.load();
    d["h2_data_frames"] = s.h2_send.data_frames.load();
    d["h2_queue_wait_us"] = s.h2_send.queue_wait_ns.load() / 1000;
    d["h2_queue_wait_max_us"] = s.h2_send.queue_wait_max_ns.load() / 1000;
    d["h2_responses"] = s.h2_responses.load();
    d["h2_ttfb_us"] = s.h2_ttfb_ns.load() / 1000;
    d["h2_ttfb_max_us"] = s.h2_ttfb_max_ns.load() / 1000;
    return d;
  }
  std::string issue_token() { return srv_->issue_token(); }

 private:
  std::shared_ptr<ObjectStore> store_;
  std::unique_ptr<FakeGcsServer> srv_;
};

const CrcTables& host_tables() {
  static CrcTables* t = [] {
    auto* x = new CrcTables();
    build_crc_tables(x);
    return x;
  }();
  return *t;
}

}  // namespace

namespace {
// An exception escaping a native thread (or thrown during unwinding) ends the
// process in std::terminate.  Under pytest, stderr is captured at the fd
// level, so the runtime's own message is lost with the process: write the
// exception, the thread and a backtrace straight to the terminal's stderr.
std::terminate_handler g_prev_terminate = nullptr;

[[noreturn]] void terminate_with_report() {
  char name[32] = "?";
  pthread_getname_np(pthread_self(), name, sizeof(name));
  std::string what = "(no active exception)";
  if (std::exception_ptr ep = std::current_exception()) {
    try {
      std::rethrow_exception(ep);
    } catch (const std::exception& e) {
      what = std::string(typeid(e).name()) + ": " + e.what();
    } catch (...) {
      what = "(non-std exception)";
    }
  }
  const std::string head = "gcsb: std::terminate in thread '" + std::string(name) + "': " + what + "\n";
  void* frames[64];
  const int nf = backtrace(frames, 64);
  (void)!::write(2, head.data(), head.size());
  backtrace_symbols_fd(frames, nf, 2);
  if (const char* path = std::getenv("GCSB_TERMINATE_LOG"); path && *path) {
    const int lf = ::open(path, O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    if (lf >= 0) {
      (void)!::write(lf, head.data(), head.size());
      backtrace_symbols_fd(frames, nf, lf);
      ::close(lf);
    }
  }
  if (g_prev_terminate) g_prev_terminate();  // whatever handler was installed before ours
  std::abort();
}
}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "MI355X-native object-storage benchmark core (C++/HIP)";
  // opt-in (GCSB_TERMINATE_LOG=<file>): a process-wide terminate handler is
  // no side effect an import should have; it reports to fd 2 and
  // the file, then chains to the handler it replaced
  if (const char* e = std::getenv("GCSB_TERMINATE_LOG"); e && *e) g_prev_terminate = std::set_terminate(terminate_with_report);
  py::register_exception<StorageError>(m, "StorageError");

  m.def("set_deferred_wake_blocks", [](int n) { DiscardSink::wake_blocks().store(n); },
        "A/B: a deferred discard sink wakes its worker once this many blocks are queued (0: every message)");

  m.def("crc32c", [](const py::bytes& b) {
    std::string s = b;
    return gcsb::crc32c(s.data(), s.size());
  });
  m.def("crc32c_extend", [](uint32_t crc, const py::bytes& b) {
    std::string s = b;
    return crc32c_extend(crc, s.data(), s.size());
  });
  m.def("crc32c_combine", &crc32c_combine);
  m.def("crc32c_shift", &crc32c_shift);
  m.def("crc32c_fixup", &crc32c_fixup);
  m.def("crc32c_raw", [](const py::bytes& b) {
    std::string s = b;
    return crc32c_raw_update(0, s.data(), s.size());
  });
  m.def("crc32c_hw_available", &crc32c_hw_available);
  m.def(
      "emulate_gpu_crc32c",
      [](const py::bytes& b, size_t misalign, uint32_t expected, bool check, uint32_t tile_log2, int fold_waves) {
        std::string s = b;
        std::vector<uint8_t> buf(s.size() + 64);
        uint8_t* base = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(buf.data()) + 15) & ~uintptr_t(15));
        uint8_t* p = base + (misalign % 16);
        std::memcpy(p, s.data(), s.size());
        if (tile_log2 != kCrcMinTileLog2 && tile_log2 != kCrcMaxTileLog2)
          throw std::invalid_argument("tile_log2 must be 12 or 14");
        if (fold_waves != 0 && fold_waves != 1 && fold_waves != 8)
          throw std::invalid_argument("fold_waves must be 0 (slot kernel), 1 or 8");
        CrcSegResult r = emulate_crc32c_segment(p, static_cast<uint32_t>(s.size()), host_tables(), expected, check,
                                                tile_log2, fold_waves);
        return py::make_tuple(r.raw, r.crc, r.status);
      },
      py::arg("data"), py::arg("misalign") = 0, py::arg("expected") = 0, py::arg("check") = false,
      py::arg("tile_log2") = kCrcMaxTileLog2, py::arg("fold_waves") = 8);
  m.def("object_rotation", &object_rotation);
  m.def("object_bytes", [](const std::string& name, uint64_t off, uint64_t n) {
    std::string out(n, '\0');
    fill_object_bytes(reinterpret_cast<uint8_t*>(&out[0]), object_rotation(name), off, n);
    return py::bytes(out);
  });
  m.def("object_crc32c", [](const std::string& name, uint64_t off, uint64_t n) {
    return PatternBuffer::instance().crc32c_range(object_rotation(name), off, n);
  });
  m.def("pattern_len", [] { return kPatternLen; });
  m.def("oc_latency_bounds_ms", [] {
    return std::vector<double>(kOcLatencyBoundsMs, kOcLatencyBoundsMs + 34);
  });
  m.def("oc_bucket_index", &oc_bucket_index);
  m.def("base64_encode", [](const py::bytes& b) { return base64_encode(std::string(b)); });
  m.def("parse_goog_hash", [](const std::string& v) {
    bool has = false;
    uint32_t crc = 0;
    std::string md5;
    parse_goog_hash(v, &has, &crc, &md5);
    return py::make_tuple(has, crc, py::bytes(md5));
  });

  // HTTP/2 + protobuf codecs (exposed for interop / conformance tests)
  m.attr("HAS_GRPC") = true;
  m.def("huffman_encode", [](const py::bytes& b) { return py::bytes(huffman_encode(std::string(b))); });
  m.def("huffman_decode", [](const py::bytes& b) {
    std::string s = b, out;
    if (!huffman_decode(reinterpret_cast<const uint8_t*>(s.data()), s.size(), &out))
      throw std::runtime_error("bad huffman string");
    return py::bytes(out);
  });
  m.def(
      "hpack_encode",
      [](const std::vector<std::pair<std::string, std::string>>& h, bool huffman) {
        std::string out;
        HpackEncoder(huffman).encode(h, &out);
        return py::bytes(out);
      },
      py::arg("headers"), py::arg("huffman") = false);
  m.def("hpack_decode_blocks", [](const std::vector<py::bytes>& blocks) {
    HpackDecoder d;
    std::vector<std::vector<std::pair<std::string, std::string>>> out;
    for (const auto& b : blocks) {
      std::string s = b;
      HeaderList hl;
      d.decode(reinterpret_cast<const uint8_t*>(s.data()), s.size(), &hl);
      out.push_back(hl);
    }
    return out;
  });
  m.def("pb_read_request", [](const std::string& bucket, const std::string& object, int64_t off, int64_t lim) {
    v2::ReadObjectRequest q;
    q.bucket = v2::bucket_resource(bucket);
    q.object = object;
    q.read_offset = off;
    q.read_limit = lim;
    return py::bytes(v2::encode_read_request(q));
  });
  m.def("pb_read_response", [](const py::bytes& content, uint32_t crc, uint32_t obj_crc, int64_t size,
                               const std::string& name) {
    std::string c = content;
    std::string cs = v2::encode_checksums(true, obj_crc, "");
    v2::Object o;
    o.name = name;
    o.size = size;
    o.bucket = "projects/_/buckets/b";
    std::string meta = v2::encode_object(o);
    v2::ContentRange cr;
    cr.end = size;
    cr.complete_length = size;
    std::string rg = v2::encode_content_range(cr);
    v2::ReadResponseFrame f = v2::encode_read_response(c.size(), true, crc, &cs, &rg, &meta);
    return py::bytes(f.head + c + f.tail);
  });
  m.def("pb_write_request", [](const std::string& upload_id, const std::string& bucket, const std::string& name,
                               int64_t off, const py::bytes& content, bool finish, uint32_t obj_crc) {
    std::string c = content;
    v2::WriteObjectSpec spec;
    spec.resource.name = name;
    spec.resource.bucket = v2::bucket_resource(bucket);
    std::string sp = v2::encode_write_spec(spec);
    std::string cs = v2::encode_checksums(true, obj_crc, "");
    v2::WriteRequestParts p = v2::encode_write_request(upload_id, upload_id.empty() ? &sp : nullptr, off, c.size(),
                                                       true, crc32c(c.data(), c.size()), finish ? &cs : nullptr,
                                                       finish);
    return py::bytes(p.head + c + p.tail);
  });
  m.def("pb_decode_object", [](const py::bytes& b) {
    v2::Object o;
    if (!v2::decode_object(std::string(b), &o)) throw std::runtime_error("bad Object");
    py::dict d;
    d["name"] = o.name;
    d["bucket"] = o.bucket;
    d["size"] = o.size;
    d["generation"] = o.generation;
    d["crc32c"] = o.crc32c;
    d["has_crc32c"] = o.has_crc32c;
    d["content_type"] = o.content_type;
    return d;
  });

  m.def("rsa_generate", [] {
    std::string a, b;
    rsa_generate_pem(&a, &b);
    return py::make_tuple(a, b);
  });
  m.def("get_access_token", [](const std::string& key_file, const std::string& token_uri) {
    py::gil_scoped_release nogil;
    auto ts = get_token_source(key_file, kScopeFullControl, token_uri);
    return std::make_pair(ts->kind(), ts->token());
  });
  m.def("service_account_assertion", [](const std::string& key_json, const std::string& token_uri, int64_t now_s) {
    ServiceAccountTokenSource ts(key_json, kScopeFullControl, token_uri);
    return ts.build_assertion(now_s);
  });

  // GPU
  m.def("gpu_device_count", &gpu_device_count);
  m.def("gpu_pci_bus_id", [](int dev) {
    char buf[64] = {0};
    hip_check(hipDeviceGetPCIBusId(buf, sizeof(buf), dev), "hipDeviceGetPCIBusId");
    return std::string(buf);
  });
  m.def("parse_cpulist", &parse_cpulist);
  m.def("pin_current_thread", &pin_current_thread);
  m.def("set_submitter_cpus", &set_submitter_cpus);
  m.def("set_submitter_spin_us", &set_submitter_spin_us, py::arg("us"));
  m.def("reserve_fd_table", &reserve_fd_table, py::arg("slots") = 8192);
  m.def("recv_stats", [] {
    RecvStats r = recv_stats();
    return py::make_tuple(r.calls, r.bytes);
  });
  m.def("recv_diag", [] {
    RecvStats r = recv_stats();
    py::dict d;
    d["calls"] = r.diag_calls;
    d["empty"] = r.diag_empty;
    d["short"] = r.diag_short;
    d["inq_bytes"] = r.diag_inq_bytes;
    d["want_bytes"] = r.diag_want_bytes;
    d["recv_ns"] = r.diag_recv_ns;
    return d;
  });
  m.def("thp_bytes_of", [](uintptr_t p, size_t n) { return thp_bytes_of(reinterpret_cast<const void*>(p), n); });
  m.def("h2_reader_stats", [] {
    H2ReaderStats s = h2_reader_stats();
    py::dict d;
    d["frames"] = s.frames;
    d["data_frames"] = s.data_frames;
    d["header_blocks"] = s.header_blocks;
    d["data_bytes"] = s.data_bytes;
    d["header_wait_ns"] = s.header_wait_ns;
    d["data_ns"] = s.data_ns;
    d["headers_ns"] = s.headers_ns;
    d["other_ns"] = s.other_ns;
    d["long_waits"] = s.long_waits;
    d["long_wait_ns"] = s.long_wait_ns;
    d["spanned_frames"] = s.spanned_frames;
    d["span_reads"] = s.span_reads;
    d["span_spills"] = s.span_spills;
    d["readers_alive"] = s.readers_alive;
    return d;
  });
  m.def("slow_hip_calls", [] {
    SlowHipCalls s = slow_hip_calls();
    py::dict d;
    d["calls"] = s.calls;
    d["slow"] = s.slow;
    d["slow_ms_total"] = s.slow_ms_total;
    d["max_ms"] = s.max_ms;
    d["max_call"] = s.max_call;
    return d;
  });
  m.def("reset_slow_hip_calls", &reset_slow_hip_calls);
  m.def("copy_ceiling", [](int dev, const std::string& dir, size_t total, size_t chunk, int slots, int streams,
                           int iters) {
    CopyCeiling c;
    {
      py::gil_scoped_release nogil;
      c = copy_ceiling(dev, dir == "h2d", total, chunk, slots, streams, iters);
    }
    py::dict d;
    d["gbps"] = c.gbps;
    d["pass_ms_p50"] = c.pass_ms_p50;
    return d;
  }, py::arg("device"), py::arg("dir") = "h2d", py::arg("total") = size_t(256) << 20, py::arg("chunk") = size_t(2) << 20,
     py::arg("slots") = 8, py::arg("streams") = 8, py::arg("iters") = 5);
  m.def("loopback_ceiling", [](const py::dict& d) {
    // upload bound (blocks.py write block): the sender sends a GpuByteSource's
    // staging pages -- HBM copied D2H into pinned slots, as a timed upload --
    // instead of the endpoint's THP object
    struct GpuStaged : CeilingSource {
      int dev;
      const void* p;
      uint64_t n;
      size_t slot;
      int slots;
      std::unique_ptr<GpuByteSource> src;
      GpuStaged(int d, const void* ptr, uint64_t bytes, size_t sb, int ns)
          : dev(d), p(ptr), n(bytes), slot(sb), slots(ns) {}
      void begin() override { src = std::make_unique<GpuByteSource>(dev, p, n, slot, slots, true, true); }
      std::pair<const uint8_t*, size_t> next(size_t max) override { return src->next(max); }
      void end() override { src.reset(); }
    };
    CeilingConfig c;
    c.object_bytes = get_or<size_t>(d, "object_bytes", c.object_bytes);
    c.reads = get_or<int>(d, "reads", c.reads);
    c.ring_bytes = get_or<size_t>(d, "ring_bytes", c.ring_bytes);
    c.recv_chunk = get_or<size_t>(d, "recv_chunk", c.recv_chunk);
    c.rcvbuf = get_or<int>(d, "rcvbuf", 0);
    c.zerocopy_send = get_or<bool>(d, "zerocopy_send", true);
    c.thp_source = get_or<bool>(d, "thp_source", true);
    c.ring_pages = get_or<int>(d, "ring_pages", 1);
    if (d.contains("send_cpus")) c.send_cpus = d["send_cpus"].cast<std::vector<int>>();
    if (d.contains("recv_cpus")) c.recv_cpus = d["recv_cpus"].cast<std::vector<int>>();
    const std::string mode = get_or<std::string>(d, "mode", "tcp");
    std::unique_ptr<GpuStaged> staged;
    if (d.contains("gpu_source_ptr")) {
      staged = std::make_unique<GpuStaged>(get_or<int>(d, "gpu_source_device", 0),
                                           reinterpret_cast<const void*>(d["gpu_source_ptr"].cast<uintptr_t>()),
                                           c.object_bytes, get_or<size_t>(d, "gpu_source_slot_bytes", size_t(2) << 20),
                                           get_or<int>(d, "gpu_source_slots", 4));
      c.source = staged.get();
    }
    CeilingResult r;
    {
      py::gil_scoped_release nogil;
      r = mode == "memcpy" ? memcpy_ceiling(c) : tcp_ceiling(c);
    }
    py::dict o;
    o["gbps"] = r.gbps;
    o["p50_ms"] = r.p50_ms;
    o["recv_cpu_s_per_gib"] = r.recv_cpu_s_per_gib;
    o["send_cpu_s_per_gib"] = r.send_cpu_s_per_gib;
    return o;
  });
  m.def("warm_copy_engines", [](int dev) {
    py::gil_scoped_release nogil;
    return warm_copy_engines(dev);
  });
  m.def("copy_engine_probe", [](int dev) {
    py::gil_scoped_release nogil;
    return copy_engine_probe(dev);
  });
  m.def("warm_device_streams", [](int dev) {
    py::gil_scoped_release nogil;
    warm_device_streams(dev);
  });
  m.def("numa_nodes_of", [](uintptr_t p, size_t n) { return numa_nodes_of(reinterpret_cast<const void*>(p), n); });
  m.def("pattern_memfd_numa", [] { return PatternBuffer::instance().memfd_numa(); });
  m.def("current_numa_node", &current_numa_node);
  m.def("gpu_crc32c", [](int dev, uintptr_t ptr, size_t n) {
    py::gil_scoped_release nogil;
    return gpu_crc32c(dev, reinterpret_cast<const void*>(ptr), n);
  });
  m.def("gpu_fill_pattern", [](int dev, uintptr_t ptr, uint64_t n, const std::string& name, uint64_t off) {
    py::gil_scoped_release nogil;
    gpu_fill_pattern(dev, reinterpret_cast<void*>(ptr), n, object_rotation(name), off);
  });
  m.def(
      "gpu_crc32c_throughput",
      [](int dev, uintptr_t ptr, size_t n, int iters, size_t seg_bytes, int tile_log2, uint32_t probe) {
        uint32_t c0 = 0;
        double gbs;
        {
          py::gil_scoped_release nogil;
          gbs = gpu_crc32c_throughput(dev, reinterpret_cast<const void*>(ptr), n, iters, seg_bytes, &c0, tile_log2,
                                      probe);
        }
        return py::make_tuple(gbs, c0);
      },
      py::arg("device"), py::arg("ptr"), py::arg("n"), py::arg("iters") = 20, py::arg("seg_bytes") = 64u << 20,
      py::arg("tile_log2") = 0, py::arg("probe") = 0);
  // CRC kernel variant selection (gpu/crc32c_gpu.h CrcLaunchOptions), for
  // kernel A/Bs and tests; returns the options now in force
  m.def("set_crc_options", [](const py::dict& d) {
    CrcLaunchOptions o = crc_launch_options();
    o.slot_waves = get_or<int>(d, "slot_waves", o.slot_waves);
    o.xor_arrival = get_or<bool>(d, "xor_arrival", o.xor_arrival);
    o.slice8 = get_or<bool>(d, "slice8", o.slice8);
    o.bank_private = get_or<bool>(d, "bank_private", o.bank_private);
    set_crc_launch_options(o);
    py::dict r;
    r["bank_private"] = o.bank_private;
    r["slot_waves"] = o.slot_waves;
    r["xor_arrival"] = o.xor_arrival;
    r["slice8"] = o.slice8;
    return r;
  }, py::arg("options") = py::dict());
  m.def("gpu_read_bytes",[](int dev, uintptr_t ptr, size_t n) {
    std::string out(n, '\0');
    {
      py::gil_scoped_release nogil;
      hip_check(hipSetDevice(dev), "hipSetDevice");
      hip_check(hipMemcpy(&out[0], reinterpret_cast<const void*>(ptr), n, hipMemcpyDeviceToHost), "hipMemcpy");
    }
    return py::bytes(out);
  });
  m.def("gpu_verify_pattern",[](int dev, uintptr_t ptr, uint64_t n, const std::string& name, uint64_t off) {
    uint64_t first = 0, bad = 0;
    {
      py::gil_scoped_release nogil;
      bad = gpu_verify_pattern(dev, reinterpret_cast<const void*>(ptr), n, object_rotation(name), off, &first);
    }
    return py::make_tuple(bad, first);
  });

  py::class_<PySlicedWriter>(m, "SlicedWriter")
      .def(py::init<const py::dict&>())
      .def("write_bytes", &PySlicedWriter::write_bytes, py::arg("bucket"), py::arg("name"), py::arg("data"),
           py::arg("resumable") = true, py::arg("chunk_bytes") = 16u << 20)
      .def("write_from_device", &PySlicedWriter::write_from_device, py::arg("bucket"), py::arg("name"),
           py::arg("dptr"), py::arg("n"), py::arg("device") = 0, py::arg("resumable") = true,
           py::arg("chunk_bytes") = 16u << 20, py::arg("slot_bytes") = 8u << 20, py::arg("slots") = 4,
           py::arg("async_stage") = true);

  py::class_<PySlicedGpuReader>(m, "SlicedGpuReader")
      .def(py::init<const py::dict&>())
      .def("read_into", &PySlicedGpuReader::read_into, py::arg("bucket"), py::arg("name"), py::arg("dptr"),
           py::arg("n"));

  py::class_<PyGpuSink>(m, "GpuSink")
      .def(py::init([](const py::dict& d) {
        auto* s = new PyGpuSink();
        s->sink = std::make_unique<GpuSink>(gpu_from(d));
        return s;
      }))
      .def("set_external_destination",
           [](PyGpuSink& s, uintptr_t ptr, size_t cap) { s.sink->set_external_destination(reinterpret_cast<void*>(ptr), cap); })
      .def_property_readonly("device_ptr", [](PyGpuSink& s) { return reinterpret_cast<uintptr_t>(s.sink->object_device_ptr()); })
      .def_property_readonly("capacity", [](PyGpuSink& s) { return s.sink->object_capacity(); })
      .def("stats", [](PyGpuSink& s) { return gpu_stats_dict(s.sink->stats()); })
      .def("ring_numa", [](PyGpuSink& s) {
        // per ring slot: pages by NUMA node (affinity.h numa_nodes_of)
        py::list out;
        for (const auto& [p, n] : s.sink->ring_ranges()) out.append(numa_nodes_of(p, n));
        return out;
      });

  py::class_<PyClient>(m, "Client")
      .def(py::init<const py::dict&>())
      .def("read", &PyClient::read, py::arg("bucket"), py::arg("name"), py::arg("sink") = "discard",
           py::arg("host_crc") = true, py::arg("offset") = 0, py::arg("limit") = -1)
      .def("read_gpu", &PyClient::read_gpu, py::arg("bucket"), py::arg("name"), py::arg("sink"), py::arg("offset") = 0,
           py::arg("limit") = -1)
      .def("read_bytes", &PyClient::read_bytes, py::arg("bucket"), py::arg("name"), py::arg("offset") = 0,
           py::arg("limit") = -1)
      .def("stat", &PyClient::stat)
      .def("list", &PyClient::list, py::arg("bucket"), py::arg("prefix") = "", py::arg("page_size") = 1000,
           py::arg("page_token") = "", py::arg("delimiter") = "")
      .def("list_all", &PyClient::list_all, py::arg("bucket"), py::arg("prefix") = "", py::arg("page_size") = 1000)
      .def("write_bytes", &PyClient::write_bytes, py::arg("bucket"), py::arg("name"), py::arg("data"),
           py::arg("resumable") = true, py::arg("chunk_bytes") = 16u << 20)
      .def("write_from_device", &PyClient::write_from_device, py::arg("bucket"), py::arg("name"), py::arg("dptr"),
           py::arg("n"), py::arg("device") = 0, py::arg("resumable") = true, py::arg("chunk_bytes") = 16u << 20,
           py::arg("slot_bytes") = 8u << 20, py::arg("slots") = 4, py::arg("async_stage") = true)
      .def("compose", &PyClient::compose, py::arg("bucket"), py::arg("dest"), py::arg("sources"),
           py::arg("content_type") = "")
      .def("last_upload",
           [](PyClient& c) {
             const UploadPhases ph = c.client().last_upload();
             py::dict p;
             p["start_rpc_ms"] = ph.start_rpc_ns / 1e6;
             p["first_send_ms"] = ph.first_send_ns / 1e6;
             p["last_send_ms"] = ph.last_send_ns / 1e6;
             p["response_ms"] = ph.response_ns / 1e6;
             return p;
           },
           "the last finished upload's phases, ms from its start (gRPC; 0 = not reached)")
      .def("delete", &PyClient::remove)
      .def("stats", &PyClient::stats);

  m.attr("LOOPBACK_RTO_MIN_US") = kLoopbackRtoMinUs;
  py::class_<LatencySeries>(m, "LatencySeries")
      .def(py::init<>())
      .def("add", &LatencySeries::add)
      .def("extend", [](LatencySeries& l, const std::vector<double>& v) {
        for (double x : v) l.add(x);
      })
      .def("pct_floor", &LatencySeries::pct_floor)
      .def("__len__", &LatencySeries::size)
      .def_property_readonly("exact", &LatencySeries::exact)
      .def_property_readonly("min", &LatencySeries::min)
      .def_property_readonly("max", &LatencySeries::max)
      .def_readonly_static("EXACT_CAP", &LatencySeries::kExact);
  py::class_<PyRunner>(m, "Runner")
      .def(py::init<const py::dict&>())
      .def("start", &PyRunner::start)
      .def("wait", &PyRunner::wait)
      .def("stop", &PyRunner::stop)
      .def("drain", &PyRunner::drain)
      .def("summary", &PyRunner::summary, py::arg("percentiles") = true,
           "percentiles=False: counts, bytes, mean and the OpenCensus buckets only (O(1), for periodic exporters)")
      .def("object_for", &PyRunner::object_for)
      .def("landing_ptr", &PyRunner::landing_ptr)
      .def("ring_numa", &PyRunner::ring_numa)
      .def("ring_thp_fraction", &PyRunner::ring_thp_fraction)
      .def("conn_ring_stats", &PyRunner::conn_ring_stats,
           "counters of the multiplexed connection's shared receive ring (None without one)")
      .def("transport_path", &PyRunner::transport_path)
      .def("set_reads_per_worker", &PyRunner::set_reads_per_worker)
      .def("set_recording", &PyRunner::set_recording,
           "False: the next runs' reads are untimed (counted nowhere; a failure still counts as an error)")
      .def("reset_stats", &PyRunner::reset_stats);

  py::class_<PyServer>(m, "Server")
      .def(py::init<const py::dict&>())
      .def("start", &PyServer::start)
      .def("stop", &PyServer::stop)
      .def_property_readonly("port", &PyServer::port)
      .def_property_readonly("url", &PyServer::url)
      .def("add_synthetic", &PyServer::add_synthetic, py::arg("bucket"), py::arg("prefix"), py::arg("suffix") = "",
           py::arg("first") = 0, py::arg("count") = 1, py::arg("size") = 1 << 20)
      .def("add_object", &PyServer::add_object)
      .def("object_info", &PyServer::object_info)
      .def("object_bytes", &PyServer::object_bytes)
      .def("set_faults", &PyServer::set_faults)
      .def("stats", &PyServer::stats)
      .def("issue_token", &PyServer::issue_token);
}
