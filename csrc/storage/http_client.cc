// HTTP transport for the storage client: XML API media reads (the library's
// default read path), JSON API reads (alt=media), JSON
// metadata/list, and resumable / single-request uploads.
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>

#include "core/json.h"
#include "core/util.h"
#include "h2/h2_client.h"
#include "http1/http1.h"
#include "storage/client.h"

namespace gcsb {
namespace {

SocketOptions with_alpn(SocketOptions o, const char* alpn) {
  o.alpn = alpn;
  return o;
}

bool http_retryable(int status) { return status == 408 || status == 429 || status >= 500; }

ObjectMeta meta_from_json(const Json& j) {
  ObjectMeta m;
  m.name = j.get_string("name");
  m.bucket = j.get_string("bucket");
  m.size = j.get_int("size");
  m.generation = j.get_int("generation");
  m.metageneration = j.get_int("metageneration", 1);
  if (const Json* c = j.get("crc32c"); c && c->is_string()) m.has_crc32c = crc32c_from_b64(c->as_string(), &m.crc32c);
  if (const Json* h = j.get("md5Hash"); h && h->is_string()) base64_decode(h->as_string(), &m.md5);
  m.content_type = j.get_string("contentType");
  m.updated = j.get_string("updated");
  return m;
}

[[noreturn]] void throw_status(int status, const std::string& what, const std::string& body) {
  std::string msg = what + ": HTTP " + std::to_string(status);
  if (!body.empty()) msg += ": " + body.substr(0, 512);
  if (status == 404) msg = "storage: object doesn't exist (" + what + ")";
  throw StorageError(msg, http_retryable(status), status);
}

// ObjectInfo of a media response from its headers (name -> value lookups are
// case-insensitive: HTTP/1.1 names as sent, HTTP/2 names lower-case).
template <typename Get, typename Each>
ObjectInfo media_info(int status, int64_t content_length, int64_t offset, Get get, Each each_hash) {
  ObjectInfo info;
  info.start_offset = offset;
  if (const std::string* g = get("x-goog-generation")) info.generation = std::stoll(*g);
  each_hash([&](const std::string& v) { parse_goog_hash(v, &info.has_crc32c, &info.crc32c, &info.md5); });
  if (status == 206) {
    if (const std::string* cr = get("content-range")) {
      size_t slash = cr->find('/');
      if (slash != std::string::npos && (*cr)[slash + 1] != '*') info.size = std::stoll(cr->substr(slash + 1));
    }
  } else if (content_length >= 0) {
    info.size = content_length;
  }
  if (const std::string* sl = get("x-goog-stored-content-length"); sl && info.size < 0) info.size = std::stoll(*sl);
  return info;
}

// One media GET on an HTTP/2 stream.  The connection's reader thread hands
// DATA to it on the socket, so body bytes are recv()'d straight into the sink
// window (one copy, as on HTTP/1.1 and gRPC).  Sink errors are recorded and
// the rest of the body skipped; the caller rethrows after completion.
class H2MediaGet : public H2ClientStream {
 public:
  H2MediaGet(Sink& sink, ReadResult* rr, uint64_t* delivered, int64_t offset, int64_t limit, bool first_attempt)
      : sink_(sink), rr_(rr), delivered_(delivered), offset_(offset), limit_(limit), first_(first_attempt),
        cap_total_(limit >= 0 ? *delivered + static_cast<uint64_t>(limit) : ~0ull) {}

  void on_headers(const HeaderList& h, bool end_stream) override {
    if (!got_head_) {
      got_head_ = true;
      int64_t clen = -1;
      for (const auto& kv : h) {
        if (kv.first == ":status") status_ = std::atoi(kv.second.c_str());
        if (kv.first == "content-length") clen = std::strtoll(kv.second.c_str(), nullptr, 10);
      }
      if (status_ == 200 || status_ == 206) {
        auto get = [&](const char* n) -> const std::string* {
          for (const auto& kv : h)
            if (kv.first == n) return &kv.second;
          return nullptr;
        };
        auto each = [&](auto&& f) {
          for (const auto& kv : h)
            if (kv.first == "x-goog-hash") f(kv.second);
        };
        try {
          ObjectInfo info = media_info(status_, clen, offset_, get, each);
          // server ignored Range: skip what we already have, as the HTTP/1.1
          // path does (an error here would retry forever against that server)
          if (status_ == 200 && offset_ > 0) skip_left_ = static_cast<uint64_t>(offset_);
          // body bytes bound for the sink (spanning reads stay within them)
          if (clen >= 0) body_left_ = std::max<int64_t>(0, clen - static_cast<int64_t>(skip_left_));
          const bool full = offset_ == 0 && limit_ < 0 && status_ == 200;
          if (first_) {
            ObjectInfo bi = info;
            if (!full) bi.has_crc32c = false;
            sink_.begin(bi);
            rr_->sink_begun = true;
            rr_->info = info;
          }
        } catch (const std::exception& e) {
          fail(e.what(), false);
        }
      }
    }
    if (end_stream) done();
  }

  void on_data(H2DataCursor& c) override {
    if (status_ != 200 && status_ != 206) {
      // error body (JSON / XML), kept for the message
      while (c.left() > 0) {
        char tmp[4096];
        size_t k = std::min<size_t>(c.left(), sizeof(tmp));
        c.read_exact(tmp, k);
        if (err_body_.size() < 4096) err_body_.append(tmp, k);
      }
    } else {
      while (c.left() > 0) {
        if (skip_left_ > 0) {
          const uint32_t k = static_cast<uint32_t>(std::min<uint64_t>(c.left(), skip_left_));
          c.skip(k);
          skip_left_ -= k;
          continue;
        }
        if (failed_.load() || *delivered_ >= cap_total_) {
          if (!failed_.load()) fail("http2 GET: server sent more than the requested range", false);
          c.skip(c.left());
          break;
        }
        // the body may run on past this frame: a spanning read takes the
        // frames that follow (H2DataCursor::read_spanning), up to the range
        // still expected (content-length / the requested range)
        const uint64_t expect = body_left_ > 0 ? static_cast<uint64_t>(body_left_) : c.left();
        const uint64_t want = std::max<uint64_t>(c.left(), std::min<uint64_t>(expect, cap_total_ - *delivered_));
        Window w;
        try {
          w = sink_.acquire(static_cast<size_t>(want));
        } catch (const std::exception& e) {
          fail(std::string("sink: ") + e.what(), false);
          continue;
        }
        size_t cap = static_cast<size_t>(std::min<uint64_t>({want, w.cap, cap_total_ - *delivered_}));
        size_t m = c.read_spanning(w.ptr, cap);
        if (body_left_ > 0) body_left_ -= static_cast<int64_t>(std::min<uint64_t>(m, body_left_));
        if (!rr_->first_byte_ns) rr_->first_byte_ns = now_ns();
        try {
          sink_.commit(m);
        } catch (const std::exception& e) {
          fail(std::string("sink: ") + e.what(), false);
        }
        *delivered_ += m;
        // deferred sink (host CRC on the waiting worker): wake it every
        // 2 MiB so its replay overlaps the rest of the body arriving
        if (sink_.deferred() && (unpoked_ += m) >= (2u << 20)) {
          unpoked_ = 0;
          poke();
        }
      }
    }
    if (c.end_stream()) done();
  }

  void on_reset(uint32_t code) override {
    fail("http2 GET: RST_STREAM code " + std::to_string(code), true);
    done();
  }
  void on_conn_error(const std::string& msg) override {
    fail("http2 connection error: " + msg, true);
    done();
  }

  // Waits for END_STREAM / reset; returns the HTTP status, throws on
  // transport or sink errors.
  // idle_ms > 0 (-read-timeout): see GrpcCall::wait_ok -- on_idle abandons
  // the stream (H2ClientConn::abandon_stream) before the retryable timeout.
  int wait(std::string* body, int idle_ms = 0, const std::function<void()>& on_idle = {}) {
    std::unique_lock<std::mutex> lk(mu_);
    const bool drain = sink_.deferred();
    for (;;) {
      if (!wait_progress(cv_, lk, [&] { return done_ || (drain && poked_); }, idle_ms)) {
        lk.unlock();
        if (on_idle) on_idle();
        if (drain) sink_.drain();  // (see GrpcCall::wait_ok)
        throw StorageError("read timeout: no data for " + std::to_string(idle_ms) + " ms", true);
      }
      poked_ = false;
      if (!drain) break;
      const bool d = done_;
      lk.unlock();
      sink_.drain();
      lk.lock();
      if (d) break;
    }
    if (!error_.empty()) throw StorageError(error_, retryable_);
    if (!got_head_) throw StorageError("http2 GET: stream ended without a response", true);
    *body = err_body_;
    return status_;
  }

 private:
  void fail(const std::string& msg, bool retryable) {
    std::lock_guard<std::mutex> lk(mu_);
    if (error_.empty()) {
      error_ = msg;
      retryable_ = retryable;
    }
    failed_ = true;
  }
  void done() {
    std::lock_guard<std::mutex> lk(mu_);
    done_ = true;
    cv_.notify_all();
  }
  void poke() {
    std::lock_guard<std::mutex> lk(mu_);
    poked_ = true;
    cv_.notify_all();
  }
  Sink& sink_;
  ReadResult* rr_;
  uint64_t* delivered_;
  int64_t offset_, limit_;
  bool first_;
  uint64_t cap_total_;
  bool got_head_ = false;
  int status_ = 0;
  uint64_t skip_left_ = 0;  // 200 to a ranged GET: body bytes before the offset
  int64_t body_left_ = 0;   // body bytes still due for the sink (0: unknown / done)
  std::string err_body_;
  std::atomic<bool> failed_{false};
  std::mutex mu_;
  std::condition_variable cv_;
  bool done_ = false, retryable_ = false, poked_ = false;
  uint64_t unpoked_ = 0;
  std::string error_;
};

class HttpStorageClient : public StorageClient {
 public:
  explicit HttpStorageClient(const ClientConfig& cfg)
      : StorageClient(cfg),
        pool_(cfg.endpoint, with_alpn(cfg.sock, "http/1.1"), cfg.protocol == "http2" ? 0 : cfg.max_conns_per_host,
              cfg.protocol == "http2" ? 0 : cfg.max_idle_conns_per_host),
        ua_(cfg.user_agent) {
    // Decorator order mirrors the reference: oauth2.Transport wraps the base
    // transport, the User-Agent tripper wraps that (main.go:89-101).
    if (cfg.token) {
      auth_ = std::make_unique<AuthDecorator>(cfg.token);
      decorators_.push_back(auth_.get());
    }
    decorators_.push_back(&ua_);
  }

  std::string transport_name() const override { return h2_media_ ? "http2" : "http1"; }

 protected:
  std::string media_path(const std::string& bucket, const std::string& object, int64_t pin_generation) const {
    std::string path;
    if (cfg_.http_api == "json")
      path = "/storage/v1/b/" + url_encode(bucket) + "/o/" + url_encode(object) + "?alt=media";
    else
      path = "/" + bucket + "/" + url_encode(object, true);
    if (pin_generation)
      path += std::string(cfg_.http_api == "json" ? "&" : "?") + "generation=" + std::to_string(pin_generation);
    return path;
  }

  std::shared_ptr<H2ClientConn> h2_conn() {
    std::lock_guard<std::mutex> lk(h2_mu_);
    if (!h2_ || !h2_->usable()) {
      if (h2_) h2_->close();
      h2_ = H2ClientConn::dial(cfg_.endpoint, h2_opt_);
      ++stats_.dials;
    }
    return h2_;
  }

  // -client-protocol http2: the media GET on an HTTP/2 stream (h2c with prior
  // knowledge on http://, ALPN h2 on https://), all GETs of the client
  // multiplexed on one connection.  The reference's http2 transport
  // (main.go:74-81) forces HTTP/2 with keep-alives disabled; metadata, list
  // and upload requests here stay on the HTTP/1.1 pool, which runs without
  // keep-alive in this mode.
  void read_attempt_h2(const std::string& bucket, const std::string& object, Sink& sink, int64_t offset,
                       int64_t limit, bool first_attempt, ReadResult* rr, uint64_t* delivered) {
    Headers dh;
    for (RequestDecorator* d : decorators_) d->decorate(dh);
    HeaderList h = {{":method", "GET"},
                    {":scheme", cfg_.endpoint.scheme == "https" ? "https" : "http"},
                    {":path", media_path(bucket, object, rr->pin_generation)},
                    {":authority", cfg_.endpoint.host_header()}};
    for (const auto& kv : dh) h.emplace_back(to_lower(kv.first), kv.second);
    if (offset > 0 || limit >= 0) {
      std::string r = "bytes=" + std::to_string(offset) + "-";
      if (limit >= 0) r += std::to_string(offset + limit - 1);
      h.emplace_back("range", r);
    }
    h.emplace_back("x-goog-api-client", "gccl/1.33.0 gcsb-native");
    auto c = h2_conn();
    auto call = std::make_shared<H2MediaGet>(sink, rr, delivered, offset, limit, first_attempt);
    std::string body;
    int status = 0;
    try {
      c->start_stream(call, h, true);
      const int idle = cfg_.sock.io_timeout_ms;
      status = call->wait(&body, idle, [c, call, idle] { c->abandon_stream(*call, idle); });
    } catch (...) {
      c->end_stream(*call, true);
      throw;
    }
    c->end_stream(*call, false);
    if (status != 200 && status != 206) throw_status(status, "GET " + bucket + "/" + object, body);
  }

  void read_attempt(const std::string& bucket, const std::string& object, Sink& sink, int64_t offset, int64_t limit,
                    bool first_attempt, ReadResult* rr, uint64_t* delivered) override {
    if (h2_media_) return read_attempt_h2(bucket, object, sink, offset, limit, first_attempt, rr, delivered);
    Http1Exchange ex(pool_, decorators_);
    Headers h;
    if (offset > 0 || limit >= 0) {
      std::string r = "bytes=" + std::to_string(offset) + "-";
      if (limit >= 0) r += std::to_string(offset + limit - 1);
      h.emplace_back("Range", r);
    }
    h.emplace_back("x-goog-api-client", "gccl/1.33.0 gcsb-native");
    const HttpResponseHead& head = ex.send("GET", media_path(bucket, object, rr->pin_generation), h);
    if (head.status != 200 && head.status != 206) {
      std::string body = ex.read_body_string(1 << 20);
      throw_status(head.status, "GET " + bucket + "/" + object, body);
    }
    ObjectInfo info = media_info(
        head.status, head.content_length, offset, [&](const char* n) { return head.get(n); },
        [&](auto&& f) {
          for (const auto& kv : head.headers)
            if (iequals(kv.first, "x-goog-hash")) f(kv.second);
        });
    // A whole-object CRC only applies to a full read (the library skips the
    // check for ranged reads).
    bool full = offset == 0 && limit < 0 && head.status == 200;
    if (first_attempt) {
      ObjectInfo bi = info;
      if (!full) bi.has_crc32c = false;
      sink.begin(bi);
      rr->sink_begun = true;
      rr->info = info;
    }
    if (head.status == 200 && offset > 0) {
      // server ignored Range: skip what we already have
      uint8_t tmp[65536];
      int64_t skip = offset;
      while (skip > 0) {
        size_t r = ex.read_body(tmp, skip < 65536 ? static_cast<size_t>(skip) : 65536);
        if (r == 0) throw StorageError("short body while skipping", true);
        skip -= static_cast<int64_t>(r);
      }
    }
    const size_t chunk = cfg_.read_chunk;
    // ranged read: never more than `limit` bytes into the sink
    const uint64_t cap_total = limit >= 0 ? *delivered + static_cast<uint64_t>(limit) : ~0ull;
    while (!ex.body_done()) {
      if (*delivered >= cap_total) throw StorageError("GET: server sent more than the requested range", false);
      Window w = sink.acquire(chunk);
      size_t cap = w.cap < chunk ? w.cap : chunk;
      if (cap > cap_total - *delivered) cap = static_cast<size_t>(cap_total - *delivered);
      size_t r = ex.read_body(w.ptr, cap);
      if (r == 0) break;
      if (!rr->first_byte_ns) rr->first_byte_ns = now_ns();
      sink.commit(r);
      *delivered += r;
    }
    ex.close();
  }

  ObjectMeta stat_attempt(const std::string& bucket, const std::string& object) override {
    Http1Exchange ex(pool_, decorators_);
    ex.send("GET", "/storage/v1/b/" + url_encode(bucket) + "/o/" + url_encode(object), {});
    std::string body = ex.read_body_string();
    if (ex.head().status != 200) throw_status(ex.head().status, "stat " + bucket + "/" + object, body);
    ex.close();
    return meta_from_json(Json::parse(body));
  }

  ObjectMeta compose_attempt(const std::string& bucket, const std::string& dest,
                             const std::vector<std::string>& sources, const std::string& content_type) override {
    Json body = Json::object();
    Json arr = Json::array();
    for (const auto& n : sources) {
      Json e = Json::object();
      e.set("name", Json::str(n));
      arr.push(e);
    }
    body.set("sourceObjects", arr);
    Json d = Json::object();
    if (!content_type.empty()) d.set("contentType", Json::str(content_type));
    body.set("destination", d);
    const std::string b = body.dump();
    Http1Exchange ex(pool_, decorators_);
    ex.send("POST", "/storage/v1/b/" + url_encode(bucket) + "/o/" + url_encode(dest) + "/compose",
            {{"Content-Type", "application/json; charset=UTF-8"}}, b.data(), b.size());
    std::string rb = ex.read_body_string();
    if (ex.head().status != 200) throw_status(ex.head().status, "compose " + bucket + "/" + dest, rb);
    ex.close();
    return meta_from_json(Json::parse(rb));
  }

  void delete_attempt(const std::string& bucket, const std::string& object) override {
    Http1Exchange ex(pool_, decorators_);
    ex.send("DELETE", "/storage/v1/b/" + url_encode(bucket) + "/o/" + url_encode(object), {});
    std::string rb = ex.read_body_string();
    if (ex.head().status != 204 && ex.head().status != 200)
      throw_status(ex.head().status, "delete " + bucket + "/" + object, rb);
    ex.close();
  }

  ListResult list_attempt(const std::string& bucket, const std::string& prefix, int page_size,
                          const std::string& page_token, const std::string& delimiter) override {
    std::string q = "/storage/v1/b/" + url_encode(bucket) + "/o?maxResults=" + std::to_string(page_size);
    if (!prefix.empty()) q += "&prefix=" + url_encode(prefix);
    if (!page_token.empty()) q += "&pageToken=" + url_encode(page_token);
    if (!delimiter.empty()) q += "&delimiter=" + url_encode(delimiter);
    Http1Exchange ex(pool_, decorators_);
    ex.send("GET", q, {});
    std::string body = ex.read_body_string();
    if (ex.head().status != 200) throw_status(ex.head().status, "list " + bucket, body);
    ex.close();
    Json j = Json::parse(body);
    ListResult r;
    if (const Json* items = j.get("items"))
      for (const auto& it : items->items()) r.objects.push_back(meta_from_json(it));
    if (const Json* pf = j.get("prefixes"))
      for (const auto& p : pf->items()) r.prefixes.push_back(p.as_string());
    r.next_page_token = j.get_string("nextPageToken");
    return r;
  }

  ObjectMeta write_impl(const std::string& bucket, const std::string& object, ByteSource& src,
                        const WriteOptions& opt) override {
    const uint64_t total = src.size();
    Json md = Json::object();
    md.set("name", Json::str(object));
    md.set("contentType", Json::str(opt.content_type));
    // the object's CRC32C in the session's metadata when the source already
    // has it; else (a GPU source still staging) with the final chunk
    const bool crc_up_front = src.crc32c_ready();
    if (crc_up_front) md.set("crc32c", Json::str(crc32c_b64(src.crc32c())));
    auto stream_body = [&](Conn& c, uint64_t n) {
      while (n > 0) {
        auto [p, k] = src.next(n < (8u << 20) ? static_cast<size_t>(n) : (8u << 20));
        if (k == 0) throw StorageError("upload source ended early", false);
        c.write_all(p, k);
        n -= k;
      }
    };
    if (!opt.resumable) {
      return with_retry([&] {
        src.seek(0);
        Http1Exchange ex(pool_, decorators_);
        std::string q = "/upload/storage/v1/b/" + url_encode(bucket) + "/o?uploadType=media&name=" + url_encode(object);
        Headers h{{"Content-Type", opt.content_type}};
        if (src.has_crc32c()) h.emplace_back("x-goog-hash", "crc32c=" + crc32c_b64(src.crc32c()));
        ex.send_stream("POST", q, h, total, [&](Conn& c) { stream_body(c, total); });
        std::string body = ex.read_body_string();
        if (ex.head().status != 200) throw_status(ex.head().status, "upload " + object, body);
        ex.close();
        return meta_from_json(Json::parse(body));
      });
    }
    // 1) initiate the resumable session
    std::string session = with_retry([&] {
      Http1Exchange ex(pool_, decorators_);
      std::string q = "/upload/storage/v1/b/" + url_encode(bucket) + "/o?uploadType=resumable&name=" + url_encode(object);
      std::string body = md.dump();
      Headers h{{"Content-Type", "application/json; charset=UTF-8"},
                {"X-Upload-Content-Type", opt.content_type},
                {"X-Upload-Content-Length", std::to_string(total)}};
      ex.send("POST", q, h, body.data(), body.size());
      std::string rb = ex.read_body_string();
      if (ex.head().status != 200) throw_status(ex.head().status, "start resumable upload", rb);
      const std::string* loc = ex.head().get("Location");
      if (!loc) throw StorageError("resumable upload: no Location header", false);
      ex.close();
      std::string l = *loc;
      // accept absolute URLs: keep path+query
      size_t sch = l.find("://");
      if (sch != std::string::npos) {
        size_t sl = l.find('/', sch + 3);
        l = sl == std::string::npos ? "/" : l.substr(sl);
        if (!pool_.endpoint().base_path.empty() && starts_with(l, pool_.endpoint().base_path))
          l = l.substr(pool_.endpoint().base_path.size());
      }
      return l;
    });
    // 2) upload chunks; on failure query the persisted size and resume
    const uint64_t chunk = std::max<uint64_t>(256 << 10, opt.chunk_bytes / (256 << 10) * (256 << 10));
    uint64_t off = 0;
    Backoff bo(cfg_.retry);
    int64_t t0 = now_ns();
    int attempt = 0;
    for (;;) {
      try {
        uint64_t n = std::min<uint64_t>(chunk, total - off);
        bool last = off + n == total;
        std::string cr = total == 0 ? "bytes */0"
                                    : "bytes " + std::to_string(off) + "-" + std::to_string(off + n - 1) + "/" +
                                          (last ? std::to_string(total) : "*");
        Http1Exchange ex(pool_, decorators_);
        Headers h{{"Content-Range", cr}};
        if (last && !crc_up_front && src.has_crc32c()) h.emplace_back("x-goog-hash", "crc32c=" + crc32c_b64(src.crc32c()));
        src.seek(off);
        ex.send_stream("PUT", session, h, n, [&](Conn& c) { stream_body(c, n); });
        std::string body = ex.read_body_string();
        int st = ex.head().status;
        if (st == 308) {
          uint64_t persisted = 0;
          if (const auto* rg = ex.head().get("Range")) {
            size_t dash = rg->find('-');
            if (dash != std::string::npos) persisted = std::stoull(rg->substr(dash + 1)) + 1;
          }
          ex.close();
          off = persisted;
          continue;
        }
        if (st == 200 || st == 201) {
          ex.close();
          return meta_from_json(Json::parse(body));
        }
        throw_status(st, "upload chunk", body);
      } catch (const StorageError& e) {
        ++attempt;
        if (!e.retryable() || cfg_.retry.mode == RetryMode::kNever ||
            (cfg_.retry.max_attempts > 0 && attempt >= cfg_.retry.max_attempts) ||
            (cfg_.retry.max_total_s > 0 && (now_ns() - t0) / 1e9 > cfg_.retry.max_total_s))
          throw;
        ++stats_.retries;
        sleep_seconds(bo.pause());
        // query persisted size
        try {
          Http1Exchange ex(pool_, decorators_);
          ex.send("PUT", session, {{"Content-Range", "bytes */" + std::to_string(total)}});
          std::string body = ex.read_body_string();
          if (ex.head().status == 200 || ex.head().status == 201) {
            ex.close();
            return meta_from_json(Json::parse(body));
          }
          uint64_t persisted = 0;
          if (const auto* rg = ex.head().get("Range")) {
            size_t dash = rg->find('-');
            if (dash != std::string::npos) persisted = std::stoull(rg->substr(dash + 1)) + 1;
          }
          ex.close();
          off = persisted;
        } catch (const StorageError&) {
          // keep `off`; next loop iteration retries
        }
      }
    }
  }

 private:
  Http1Pool pool_;
  const bool h2_media_ = cfg_.protocol == "http2";
  H2ClientOptions h2_opt_ = [this] {
    H2ClientOptions o;
    o.sock = with_alpn(cfg_.sock, "h2");
    o.sock.io_timeout_ms = 0;  // -read-timeout is per stream on the shared connection
    o.cpus = cfg_.reader_cpus.empty() ? cfg_.cpus : cfg_.reader_cpus;
    o.max_frame_size = cfg_.h2_max_frame_size;
    o.initial_window = cfg_.h2_window;
    o.span_max_frame = cfg_.h2_span_max_frame;
    return o;
  }();
  std::mutex h2_mu_;
  std::shared_ptr<H2ClientConn> h2_;
  UserAgentDecorator ua_;
  std::unique_ptr<AuthDecorator> auth_;
  std::vector<RequestDecorator*> decorators_;
};

}  // namespace

std::unique_ptr<StorageClient> make_http_client(const ClientConfig& cfg) {
  return std::make_unique<HttpStorageClient>(cfg);
}

}  // namespace gcsb
