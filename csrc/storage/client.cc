#include "storage/client.h"

#include <cstring>

#include "core/crc32c.h"
#include "core/util.h"

namespace gcsb {

HostByteSource::HostByteSource(const uint8_t* p, uint64_t n, bool compute_crc)
    : p_(p), n_(n), has_crc_(compute_crc) {
  if (compute_crc) crc_ = gcsb::crc32c(p, n);
}

std::pair<const uint8_t*, size_t> HostByteSource::next(size_t max) {
  uint64_t left = n_ - off_;
  size_t k = left < max ? static_cast<size_t>(left) : max;
  const uint8_t* q = p_ + off_;
  off_ += k;
  return {q, k};
}

bool should_retry(const RetryPolicy& p, const StorageError& e, int attempt, int64_t t0) {
  if (p.mode == RetryMode::kNever || !e.retryable()) return false;
  if (p.max_attempts > 0 && attempt >= p.max_attempts) return false;
  if (p.max_total_s > 0 && (now_ns() - t0) / 1e9 > p.max_total_s) return false;
  return true;
}

ReadResult StorageClient::read_object(const std::string& bucket, const std::string& object, Sink& sink,
                                      int64_t offset, int64_t limit, const volatile bool* cancel, int64_t generation,
                                      bool defer_finish) {
  ReadResult rr;
  rr.pin_generation = generation;
  uint64_t delivered = 0;
  Backoff bo(cfg_.retry);
  int64_t t0 = now_ns();
  for (int attempt = 1;; ++attempt) {
    rr.attempts = attempt;
    ++stats_.requests;
    try {
      int64_t lim = limit < 0 ? -1 : limit - static_cast<int64_t>(delivered);
      // A retry after the stream broke with every requested byte already
      // delivered (reset / GOAWAY before the trailers) has nothing left to
      // fetch: re-asking would send read_limit=0 ("to the end") over gRPC or
      // an empty Range over HTTP.  The read is complete.
      const bool nothing_left = rr.sink_begun && ((limit >= 0 && lim <= 0) ||
          (limit < 0 && rr.info.size >= 0 && offset + static_cast<int64_t>(delivered) >= rr.info.size));
      if (!nothing_left)
        read_attempt(bucket, object, sink, offset + static_cast<int64_t>(delivered), lim, !rr.sink_begun, &rr,
                   &delivered);
      rr.bytes = delivered;
      rr.host_done_ns = now_ns();
      stats_.bytes_in += delivered;
      if (!defer_finish) rr.sink = sink.finish();
      return rr;
    } catch (const StorageError& e) {
      const bool begun = rr.sink_begun;
      if (!should_retry(cfg_.retry, e, attempt, t0)) {
        if (begun) sink.abort();
        throw;
      }
      ++stats_.retries;
      if (!rr.pin_generation && rr.info.generation) rr.pin_generation = rr.info.generation;
      if (begun) sink.resume_at(offset + static_cast<int64_t>(delivered));
      sleep_seconds(bo.pause(), cancel);
      if (cancel && *cancel) {
        if (begun) sink.abort();
        throw StorageError("cancelled", false);
      }
    }
  }
}

ObjectMeta StorageClient::stat_object(const std::string& bucket, const std::string& object) {
  return with_retry([&] { return stat_attempt(bucket, object); });
}

ObjectMeta StorageClient::compose_object(const std::string& bucket, const std::string& dest,
                                        const std::vector<std::string>& sources, const std::string& content_type) {
  ++stats_.requests;
  return with_retry([&] { return compose_attempt(bucket, dest, sources, content_type); });
}

void StorageClient::delete_object(const std::string& bucket, const std::string& object) {
  ++stats_.requests;
  with_retry([&] {
    delete_attempt(bucket, object);
    return 0;
  });
}

ListResult StorageClient::list_objects(const std::string& bucket, const std::string& prefix, int page_size,
                                       const std::string& page_token, const std::string& delimiter) {
  return with_retry([&] { return list_attempt(bucket, prefix, page_size, page_token, delimiter); });
}

std::vector<ObjectMeta> StorageClient::list_all(const std::string& bucket, const std::string& prefix,
                                                int page_size) {
  std::vector<ObjectMeta> all;
  std::string tok;
  do {
    ListResult r = list_objects(bucket, prefix, page_size, tok);
    for (auto& o : r.objects) all.push_back(std::move(o));
    tok = r.next_page_token;
  } while (!tok.empty());
  return all;
}

ObjectMeta StorageClient::write_object(const std::string& bucket, const std::string& object, ByteSource& src,
                                       const WriteOptions& opt) {
  ++stats_.requests;
  ObjectMeta m = write_impl(bucket, object, src, opt);
  stats_.bytes_out += src.size();
  return m;
}

std::unique_ptr<StorageClient> make_client(const ClientConfig& cfg) {
  reserve_fd_table();  // before the first dial, off any timed path
  if (cfg.protocol == "grpc") return make_grpc_client(cfg);
  if (cfg.protocol == "http" || cfg.protocol == "http2") return make_http_client(cfg);
  throw StorageError("unknown client protocol \"" + cfg.protocol + "\" (want http|http2|grpc)", false);
}

std::string crc32c_b64(uint32_t crc) {
  uint8_t b[4];
  put_be32(b, crc);
  return base64_encode(b, 4);
}

bool crc32c_from_b64(const std::string& b64, uint32_t* crc) {
  std::string raw;
  if (!base64_decode(b64, &raw) || raw.size() != 4) return false;
  *crc = be32(reinterpret_cast<const uint8_t*>(raw.data()));
  return true;
}

void parse_goog_hash(const std::string& value, bool* has_crc, uint32_t* crc, std::string* md5) {
  for (auto part : split(value, ',')) {
    part = trim(part);
    if (starts_with(part, "crc32c=")) {
      if (crc32c_from_b64(std::string(part.substr(7)), crc)) *has_crc = true;
    } else if (starts_with(part, "md5=")) {
      std::string raw;
      if (base64_decode(part.substr(4), &raw)) *md5 = raw;
    }
  }
}

std::string format_goog_hash(uint32_t crc, const std::string& md5) {
  std::string s = "crc32c=" + crc32c_b64(crc);
  if (!md5.empty()) s += ",md5=" + base64_encode(md5);
  return s;
}

}  // namespace gcsb
