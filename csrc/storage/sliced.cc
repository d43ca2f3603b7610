#include "storage/sliced.h"

#include <algorithm>
#include <cstdio>

#include "core/affinity.h"
#include "core/crc32c.h"
#include "core/util.h"

namespace gcsb {

SlicedReader::SlicedReader(const ClientConfig& client_cfg, SlicedReadConfig cfg, MakeSink make_sink, Prepare prepare,
                           Place place)
    : cfg_(std::move(cfg)), prepare_(std::move(prepare)), place_(std::move(place)) {
  if (cfg_.slices < 1) cfg_.slices = 1;
  ClientConfig cc = client_cfg;
  cc.grpc_conn_pool_size = 1;  // one connection per slice client
  const int sinks_per_stream = cfg_.piece_bytes ? 2 : 1;
  for (int i = 0; i < cfg_.slices; ++i) {
    clients_.push_back(make_client(cc));
    for (int k = 0; k < sinks_per_stream; ++k) sinks_.push_back(make_sink(i * sinks_per_stream + k));
  }
  stream_done_ns_.assign(cfg_.slices, 0);
  jobs_.resize(cfg_.slices);
  for (int i = 1; i < cfg_.slices; ++i) threads_.emplace_back([this, i] { thread_main(i); });
}

SlicedReader::~SlicedReader() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

void SlicedReader::finish_piece(Sink& s, Piece& p) {
  try {
    p.rr.sink = s.finish();
  } catch (const std::exception& e) {
    if (p.error.empty()) p.error = e.what();
    piece_abort_ = true;
  }
}

// Piece mode: pull pieces off the shared cursor until none are left.  The
// stream alternates between its two sinks and finishes piece k (waits for its
// last slot copies + CRC kernels) only after piece k+1 has been received, so
// the copy tail of one piece overlaps the receive of the next.
void SlicedReader::run_pieces(int i) {
  const Job& j = jobs_[i];
  Sink* prev = nullptr;
  Piece* prev_piece = nullptr;
  int which = 0;
  for (;;) {
    if (piece_abort_.load() || (j.cancel && *j.cancel)) break;
    const size_t k = next_piece_.fetch_add(1);
    if (k >= pieces_.size()) break;
    Piece& p = pieces_[k];
    Sink& sk = *sinks_[2 * static_cast<size_t>(i) + static_cast<size_t>(which)];
    which ^= 1;
    bool ok = false;
    try {
      place_(i, sk, p.off, p.len);
      p.rr = clients_[i]->read_object(j.bucket, j.object, sk, static_cast<int64_t>(p.off),
                                      static_cast<int64_t>(p.len), j.cancel, j.generation, /*defer_finish=*/true);
      ok = true;
    } catch (const StorageError& e) {
      p.error = e.what();
      p.retryable = e.retryable();
    } catch (const std::exception& e) {
      p.error = e.what();
    }
    if (prev) finish_piece(*prev, *prev_piece);
    prev = nullptr;
    prev_piece = nullptr;
    if (!ok) {
      piece_abort_ = true;
      break;
    }
    prev = &sk;
    prev_piece = &p;
  }
  if (prev) finish_piece(*prev, *prev_piece);
  stream_done_ns_[static_cast<size_t>(i)] = now_ns();
}

void SlicedReader::run_slice(int i) {
  if (!pieces_.empty()) {
    run_pieces(i);
    return;
  }
  Job& j = jobs_[i];
  try {
    j.rr = clients_[i]->read_object(j.bucket, j.object, *sinks_[i], static_cast<int64_t>(j.off),
                                    static_cast<int64_t>(j.len), j.cancel, j.generation);
  } catch (const StorageError& e) {
    j.error = e.what();
    j.retryable = e.retryable();
  } catch (const std::exception& e) {
    j.error = e.what();
  }
}

void SlicedReader::thread_main(int i) {
  pin_current_thread(cfg_.cpus);
  name_current_thread("gcsb-slice");
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || jobs_[i].pending; });
    if (stop_) return;
    jobs_[i].pending = false;
    lk.unlock();
    run_slice(i);
    lk.lock();
    jobs_[i].done = true;
    done_cv_.notify_all();
  }
}

ReadResult SlicedReader::read(const std::string& bucket, const std::string& object, const volatile bool* cancel) {
  ObjectMeta m = clients_[0]->stat_object(bucket, object);
  const uint64_t total = static_cast<uint64_t>(m.size);
  prepare_(total);
  // slice boundaries on 2 MiB multiples (whole gRPC messages / ring chunks)
  int n = cfg_.slices;
  if (cfg_.min_slice_bytes) n = static_cast<int>(std::min<uint64_t>(n, std::max<uint64_t>(1, total / cfg_.min_slice_bytes)));
  const uint64_t align = 2u << 20;
  const bool piece_mode = cfg_.piece_bytes > 0 && n > 1;
  std::vector<std::pair<uint64_t, uint64_t>> ranges;
  if (piece_mode) {
    const uint64_t pb = std::max<uint64_t>(align, (cfg_.piece_bytes + align - 1) / align * align);
    const uint64_t streams = static_cast<uint64_t>(std::max(1, n));
    const uint64_t floor_b = cfg_.piece_min_bytes ? std::max<uint64_t>(align, cfg_.piece_min_bytes / align * align) : pb;
    pieces_.clear();
    for (uint64_t off = 0; off < total;) {
      uint64_t len = pb;
      if (cfg_.piece_min_bytes) {
        const uint64_t guided = ((total - off) / (2 * streams) + align - 1) / align * align;
        len = std::max(std::min(pb, guided), std::min(floor_b, pb));
      }
      Piece p;
      p.off = off;
      p.len = std::min(len, total - off);
      off += p.len;
      pieces_.push_back(std::move(p));
    }
    n = static_cast<int>(std::min<size_t>(static_cast<size_t>(n), pieces_.size()));
    next_piece_ = 0;
    piece_abort_ = false;
    std::fill(stream_done_ns_.begin(), stream_done_ns_.end(), 0);
  } else {
    uint64_t per = (total + n - 1) / std::max(1, n);
    per = (per + align - 1) / align * align;
    for (uint64_t off = 0; off < total || ranges.empty(); off += per) {
      ranges.emplace_back(off, std::min(per, total - off));
      if (total == 0) break;
    }
    n = static_cast<int>(ranges.size());
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (int i = 0; i < n; ++i) {
      Job& j = jobs_[i];
      j.bucket = bucket;
      j.object = object;
      j.cancel = cancel;
      j.generation = m.generation;  // every slice reads the stat's object version
      j.rr = ReadResult();
      j.error.clear();
      j.retryable = false;
      j.done = false;
      if (!piece_mode) {
        j.off = ranges[i].first;
        j.len = ranges[i].second;
        place_(i, *sinks_[i], j.off, j.len);
      }
      j.pending = i > 0;
    }
  }
  cv_.notify_all();
  run_slice(0);
  {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] {
      for (int i = 1; i < n; ++i)
        if (!jobs_[i].done) return false;
      return true;
    });
  }
  // merge: first error wins; otherwise combine the slice CRCs in order
  ReadResult out;
  out.info.size = m.size;
  out.info.generation = m.generation;
  out.info.has_crc32c = m.has_crc32c;
  out.info.crc32c = m.crc32c;
  out.info.md5 = m.md5;
  out.sink_begun = true;
  uint32_t crc = 0;
  bool all_verified = true;
  // parts in object order: the pieces (piece mode) or the slices
  std::vector<Piece> parts;
  int64_t first_done = 0, last_done = 0;
  for (int i = 0; i < n; ++i) {
    const int64_t d = piece_mode ? stream_done_ns_[static_cast<size_t>(i)] : jobs_[i].rr.host_done_ns;
    if (d && (!first_done || d < first_done)) first_done = d;
    if (d > last_done) last_done = d;
  }
  if (n > 1 && first_done) {
    skew_ms_sum_ += (last_done - first_done) / 1e6;
    ++reads_;
  }
  if (piece_mode) {
    parts.swap(pieces_);  // pieces_ empty again: run_slice() is in static mode unless a read sets it
  } else {
    parts.resize(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) {
      Piece& p = parts[static_cast<size_t>(i)];
      p.off = jobs_[i].off;
      p.len = jobs_[i].len;
      p.rr = jobs_[i].rr;
      p.error = jobs_[i].error;
      p.retryable = jobs_[i].retryable;
    }
  }
  const char* what = piece_mode ? "piece " : "slice ";
  for (size_t i = 0; i < parts.size(); ++i) {
    const Piece& p = parts[i];
    if (!p.error.empty())
      throw StorageError(what + std::to_string(i) + " [" + std::to_string(p.off) + ", +" + std::to_string(p.len) +
                             "): " + p.error,
                         p.retryable);
    if (p.rr.bytes != p.len) break;  // not read (cancelled): the byte count check below reports it
    out.bytes += p.rr.bytes;
    out.attempts = std::max(out.attempts, p.rr.attempts);
    if (p.rr.first_byte_ns && (!out.first_byte_ns || p.rr.first_byte_ns < out.first_byte_ns))
      out.first_byte_ns = p.rr.first_byte_ns;
    out.host_done_ns = std::max(out.host_done_ns, p.rr.host_done_ns);
    out.sink.landed_ns = std::max(out.sink.landed_ns, p.rr.sink.landed_ns);
    if (p.rr.sink.crc_mismatch && !out.sink.crc_mismatch) {
      out.sink.crc_mismatch = true;
      out.sink.detail = what + std::to_string(i) + ": " + p.rr.sink.detail;
    }
    all_verified = all_verified && p.rr.sink.verified;
    crc = crc32c_combine(crc, p.rr.sink.computed_crc32c, p.rr.bytes);
  }
  out.sink.bytes = out.bytes;
  out.sink.computed_crc32c = crc;
  if (out.bytes != total) {
    throw StorageError("sliced read: " + std::to_string(out.bytes) + " of " + std::to_string(total) + " bytes", true);
  }
  if (!cfg_.verify) {
    out.sink.verified = false;
  } else if (m.has_crc32c) {
    if (crc != m.crc32c) {
      out.sink.crc_mismatch = true;
      char b[128];
      std::snprintf(b, sizeof(b), "bad CRC on read: combined slices %08x want %08x", crc, m.crc32c);
      if (out.sink.detail.empty()) out.sink.detail = b;
    }
    out.sink.verified = !out.sink.crc_mismatch;
  } else {
    out.sink.verified = all_verified && !out.sink.crc_mismatch;
  }
  return out;
}

}  // namespace gcsb

namespace gcsb {

SlicedWriter::SlicedWriter(const ClientConfig& client_cfg, SlicedWriteConfig cfg) : cfg_(std::move(cfg)) {
  cfg_.slices = std::max(1, std::min(32, cfg_.slices));
  ClientConfig cc = client_cfg;
  cc.grpc_conn_pool_size = 1;
  for (int i = 0; i < cfg_.slices; ++i) clients_.push_back(make_client(cc));
  jobs_.resize(cfg_.slices);
  for (int i = 1; i < cfg_.slices; ++i) threads_.emplace_back([this, i] { thread_main(i); });
}

SlicedWriter::~SlicedWriter() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

void SlicedWriter::thread_main(int i) {
  pin_current_thread(cfg_.cpus);
  name_current_thread("gcsb-wslice");
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || jobs_[i].pending; });
    if (stop_) return;
    jobs_[i].pending = false;
    lk.unlock();
    try {
      jobs_[i].fn();
    } catch (const StorageError& e) {
      jobs_[i].error = e.what();
      jobs_[i].retryable = e.retryable();
    } catch (const std::exception& e) {
      jobs_[i].error = e.what();
    }
    lk.lock();
    jobs_[i].done = true;
    done_cv_.notify_all();
  }
}

// Runs jobs_[0..n) (job 0 on the caller) and waits for all of them.
void SlicedWriter::run_all(int n) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (int i = 0; i < n; ++i) {
      jobs_[i].done = false;
      jobs_[i].error.clear();
      jobs_[i].retryable = false;
      jobs_[i].pending = i > 0;
    }
  }
  cv_.notify_all();
  try {
    jobs_[0].fn();
  } catch (const StorageError& e) {
    jobs_[0].error = e.what();
    jobs_[0].retryable = e.retryable();
  } catch (const std::exception& e) {
    jobs_[0].error = e.what();
  }
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] {
    for (int i = 1; i < n; ++i)
      if (!jobs_[i].done) return false;
    return true;
  });
}

ObjectMeta SlicedWriter::write(const std::string& bucket, const std::string& object, uint64_t total,
                               const MakeSource& make_source, const WriteOptions& opt) {
  int n = cfg_.slices;
  if (cfg_.min_slice_bytes) n = static_cast<int>(std::min<uint64_t>(n, std::max<uint64_t>(1, total / cfg_.min_slice_bytes)));
  const uint64_t align = 256u << 10;  // resumable chunk granularity
  uint64_t per = (total + n - 1) / std::max(1, n);
  per = std::max<uint64_t>(align, (per + align - 1) / align * align);
  std::vector<std::pair<uint64_t, uint64_t>> parts;
  for (uint64_t off = 0; off < total || parts.empty(); off += per) {
    parts.emplace_back(off, std::min(per, total - off));
    if (total == 0) break;
  }
  n = static_cast<int>(parts.size());
  if (n == 1) {  // nothing to compose: a plain upload
    auto src = make_source(0, 0, total);
    return clients_[0]->write_object(bucket, object, *src, opt);
  }
  const std::string tag = std::to_string(wall_ns() % 1000000007) + "-" + std::to_string(++seq_);
  std::vector<std::string> names(n);
  std::vector<ObjectMeta> metas(n);
  std::vector<uint32_t> crcs(n, 0);
  std::vector<bool> has_crc(n, false);
  for (int i = 0; i < n; ++i) {
    names[i] = object + ".gcsb-part-" + tag + "-" + std::to_string(i);
    jobs_[i].fn = [&, i] {
      auto src = make_source(i, parts[i].first, parts[i].second);
      metas[i] = clients_[i]->write_object(bucket, names[i], *src, opt);
      // after the upload: a GPU source has every chunk CRC by then
      has_crc[i] = src->has_crc32c();
      crcs[i] = src->crc32c();
    };
  }
  run_all(n);
  std::string err;
  bool retryable = true;
  for (int i = 0; i < n; ++i)
    if (!jobs_[i].error.empty() && err.empty()) {
      err = "part " + std::to_string(i) + ": " + jobs_[i].error;
      retryable = jobs_[i].retryable;
    }
  auto cleanup = [&] {
    for (int i = 0; i < n; ++i)
      jobs_[i].fn = [&, i] {
        try {
          clients_[i]->delete_object(bucket, names[i]);
        } catch (const StorageError&) {
        }
      };
    run_all(n);
  };
  if (!err.empty()) {
    cleanup();
    throw StorageError("parallel composite upload of " + object + ": " + err, retryable);
  }
  ObjectMeta m = clients_[0]->compose_object(bucket, object, names, opt.content_type);
  cleanup();
  uint32_t want = 0;
  bool known = true;
  for (int i = 0; i < n; ++i) {
    known = known && has_crc[i];
    want = crc32c_combine(want, crcs[i], parts[i].second);
  }
  if (known && m.has_crc32c && m.crc32c != want) {
    char b[160];
    std::snprintf(b, sizeof(b), "composed object CRC32C %08x != combined part CRC32C %08x", m.crc32c, want);
    throw StorageError(b, false);
  }
  if (m.size != static_cast<int64_t>(total))
    throw StorageError("composed object has " + std::to_string(m.size) + " of " + std::to_string(total) + " bytes",
                       false);
  return m;
}

}  // namespace gcsb
