// gRPC transport for the storage client: google.storage.v2.Storage over the
// native HTTP/2 stack (h2c).  ReadObject responses are parsed as a stream:
// ChecksummedData.content bytes are recv()'d straight from the socket into the
// sink (pinned ring slot) with no intermediate message buffer; each message's
// crc32c is handed to the sink as a chunk boundary (checked on the GPU).
//
// Reference: CreateGrpcClient (reference main.go:106-117) — pool size 1, i.e.
// every worker's stream multiplexed on ONE connection (main.go:30,111).  The
// pool size is a flag here (--grpc-conn-pool-size), default 1.
#include <sys/uio.h>

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>

#include "core/crc32c.h"
#include "core/util.h"
#include "h2/h2_client.h"
#include "proto/storage_v2.h"
#include "proto/wire.h"
#include "storage/client.h"

namespace gcsb {
namespace {

enum GrpcCode {
  kOk = 0,
  kCancelled = 1,
  kUnknown = 2,
  kInvalidArgument = 3,
  kDeadlineExceeded = 4,
  kNotFound = 5,
  kAlreadyExists = 6,
  kPermissionDenied = 7,
  kResourceExhausted = 8,
  kFailedPrecondition = 9,
  kAborted = 10,
  kOutOfRange = 11,
  kUnimplemented = 12,
  kInternal = 13,
  kUnavailable = 14,
  kDataLoss = 15,
  kUnauthenticated = 16
};

// The storage library's ShouldRetry set for gRPC status codes [lib].
bool grpc_retryable(int code) {
  return code == kUnavailable || code == kResourceExhausted || code == kInternal || code == kDeadlineExceeded ||
         code == kUnknown;
}

int http_to_grpc(int status) {
  switch (status) {
    case 400: return kInternal;
    case 401: return kUnauthenticated;
    case 403: return kPermissionDenied;
    case 404: return kUnimplemented;
    case 429:
    case 502:
    case 503:
    case 504: return kUnavailable;
    default: return kUnknown;
  }
}

// Receives gRPC length-prefixed messages from a stream's DATA frames.
class MessageHandler {
 public:
  virtual ~MessageHandler() = default;
  virtual void begin(uint32_t len) = 0;
  // Consume 1..msg_left bytes of the current message from the DATA cursor
  // (c.left() >= 1); returns how many.  Only a spanning read
  // (H2DataCursor::read_spanning) may consume more than c.left().
  virtual uint64_t bytes(H2DataCursor& c, uint64_t msg_left) = 0;
  virtual void end() = 0;
};

class BufferingHandler : public MessageHandler {
 public:
  void begin(uint32_t len) override {
    cur_.clear();
    cur_.reserve(len);
  }
  uint64_t bytes(H2DataCursor& c, uint64_t msg_left) override {
    const size_t n = static_cast<size_t>(std::min<uint64_t>(c.left(), msg_left));
    size_t old = cur_.size();
    cur_.resize(old + n);
    c.read_exact(&cur_[old], n);
    return n;
  }
  void end() override { msgs_.push_back(std::move(cur_)); }
  std::vector<std::string>& messages() { return msgs_; }

 private:
  std::string cur_;
  std::vector<std::string> msgs_;
};

class GrpcCall : public H2ClientStream {
 public:
  explicit GrpcCall(MessageHandler* h) : handler_(h) {}

  // The reader thread dispatches into this call holding a reference to it
  // (H2ClientConn::acquire), so the end-of-stream wake can follow the unlock:
  // notified under the lock, the woken worker would block on mu_ straight
  // away and need a second wake once the reader lets go of it.
  void on_headers(const HeaderList& h, bool end_stream) override {
    {
      std::lock_guard<std::mutex> lk(mu_);
      headers_locked(h, end_stream);
    }
    if (end_stream) cv_.notify_all();
  }

  void headers_locked(const HeaderList& h, bool end_stream) {
    int http_status = 0;
    for (const auto& kv : h) {
      if (kv.first == ":status") http_status = std::atoi(kv.second.c_str());
      else if (kv.first == "grpc-status") grpc_status_ = std::atoi(kv.second.c_str());
      else if (kv.first == "grpc-message") grpc_message_ = url_decode(kv.second);
    }
    if (!got_headers_) {
      got_headers_ = true;
      if (http_status != 200 && grpc_status_ < 0) {
        grpc_status_ = http_to_grpc(http_status);
        grpc_message_ = "HTTP status " + std::to_string(http_status);
      }
    }
    if (end_stream) {
      if (grpc_status_ < 0) {
        grpc_status_ = kInternal;
        grpc_message_ = "stream ended without grpc-status";
      }
      done_ = true;
    }
  }

  void on_data(H2DataCursor& c) override {
    while (c.left() > 0) {
      if (failed_handler_) {
        c.skip(c.left());
        break;
      }
      if (have_ < 5) {
        uint32_t k = std::min<uint32_t>(c.left(), 5 - have_);
        c.read_exact(prefix_ + have_, k);
        have_ += k;
        if (have_ == 5) {
          if (prefix_[0] & 1) {
            handler_error("compressed gRPC message without negotiated encoding");
            continue;
          }
          msg_left_ = be32(prefix_ + 1);
          guarded([&] { handler_->begin(msg_left_); });
          if (msg_left_ == 0) {
            guarded([&] { handler_->end(); });
            have_ = 0;
          }
        }
        continue;
      }
      // socket errors propagate (connection level); sink errors are per call
      const uint64_t k = handler_->bytes(c, msg_left_);
      msg_left_ -= static_cast<uint32_t>(k);
      if (msg_left_ == 0) {
        guarded([&] { handler_->end(); });
        have_ = 0;
      }
    }
    if (c.end_stream()) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (grpc_status_ < 0) {
          grpc_status_ = kInternal;
          grpc_message_ = "DATA END_STREAM without trailers";
        }
        done_ = true;
      }
      cv_.notify_all();  // after the unlock, as in on_headers
    }
  }

  void on_reset(uint32_t code) override {
    std::lock_guard<std::mutex> lk(mu_);
    transport_error_ = "RST_STREAM code " + std::to_string(code);
    finish_locked();
  }

  void on_conn_error(const std::string& msg) override {
    std::lock_guard<std::mutex> lk(mu_);
    transport_error_ = "connection error: " + msg;
    finish_locked();
  }

  void handler_error(const std::string& msg) {
    failed_handler_ = true;
    std::lock_guard<std::mutex> lk(mu_);
    if (handler_error_.empty()) handler_error_ = msg;
  }

  // The reader thread has queued work for the waiting worker (a deferred
  // sink's message end): wake it.
  void poke() {
    std::lock_guard<std::mutex> lk(mu_);
    poked_ = true;
    cv_.notify_all();
  }

  // Waits for completion; throws a StorageError for any non-OK outcome.
  // sink: drained (deferred work run on this thread) at every poke and once
  // after completion.
  // idle_ms > 0 (-read-timeout): a stream silent that long has on_idle run
  // (H2ClientConn::abandon_stream: it cancels this stream alone, or closes
  // the connection if that is silent too; either way nothing writes into the
  // sink any more) and fails with a retryable "read timeout"; the read loop
  // then resumes at the delivered offset.
  void wait_ok(Sink* sink = nullptr, int idle_ms = 0, const std::function<void()>& on_idle = {}) {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      if (!wait_progress(cv_, lk, [&] { return done_ || (sink && poked_); }, idle_ms)) {
        lk.unlock();
        if (on_idle) on_idle();
        // the reader is gone: replay what it queued for this attempt, so the
        // sink's state matches the delivered offset the retry resumes at
        if (sink) sink->drain();
        throw StorageError("read timeout: no data for " + std::to_string(idle_ms) + " ms", true);
      }
      poked_ = false;
      if (!sink) break;
      const bool d = done_;
      lk.unlock();
      sink->drain();
      lk.lock();
      if (d) break;
    }
    if (!handler_error_.empty()) throw StorageError(handler_error_, handler_retryable_);
    if (!transport_error_.empty() && grpc_status_ != kOk) throw StorageError(transport_error_, true);
    if (grpc_status_ != kOk) {
      std::string m = "rpc error: code = " + std::to_string(grpc_status_) + " desc = " + grpc_message_;
      if (grpc_status_ == kNotFound) m = "storage: object doesn't exist (" + grpc_message_ + ")";
      throw StorageError(m, grpc_retryable(grpc_status_), 0, grpc_status_);
    }
  }
  bool clean() {
    std::lock_guard<std::mutex> lk(mu_);
    return done_ && transport_error_.empty() && grpc_status_ >= 0;
  }
  void set_handler_retryable(bool r) { handler_retryable_ = r; }

 private:
  template <typename F>
  void guarded(F&& f) {
    try {
      f();
    } catch (const std::exception& e) {
      handler_error(e.what());
    }
  }
  void finish_locked() {
    done_ = true;
    cv_.notify_all();
  }
  MessageHandler* handler_;
  uint8_t prefix_[5];
  uint32_t have_ = 0;
  uint32_t msg_left_ = 0;
  bool failed_handler_ = false;
  bool handler_retryable_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  bool done_ = false, got_headers_ = false, poked_ = false;
  int grpc_status_ = -1;
  std::string grpc_message_, transport_error_, handler_error_;
};

// Streaming ReadObjectResponse parser -> Sink.
class ReadObjectHandler : public MessageHandler {
 public:
  // cap: the most bytes *delivered may reach in this read (ranged reads);
  // a server sending past read_limit is a protocol error, never written into
  // the sink (a piece sink's neighbour in HBM belongs to another stream).
  ReadObjectHandler(Sink& sink, ReadResult* rr, uint64_t* delivered, bool full_read, GrpcCall** call,
                    uint64_t cap = ~0ull)
      : sink_(sink), rr_(rr), delivered_(delivered), full_read_(full_read), call_(call), cap_(cap) {}

  void begin(uint32_t len) override {
    msg_left_ = len;
    st_ = kTopTag;
    cd_left_ = 0;
    in_cd_ = false;
    content_seen_ = false;
    has_crc_ = false;
    vacc_ = 0;
    vshift_ = 0;
  }

  uint64_t bytes(H2DataCursor& c, uint64_t msg_left) override {
    uint64_t used = 0;
    while (c.left() > 0 && used < msg_left) {
      if (st_ == kContent) {
        // content may run on past this frame (a spanning read takes the
        // frames that follow); never past the message
        uint64_t k = std::min<uint64_t>(content_left_, msg_left - used);
        if (*delivered_ + std::min<uint64_t>(k, c.left()) > cap_)
          throw StorageError("ReadObject: server sent more than read_limit bytes", false);
        Window w;
        if (!sink_failed_) {
          try {
            w = sink_.acquire(static_cast<size_t>(k));
          } catch (const std::exception& e) {
            fail_sink(e.what());
          }
        }
        if (sink_failed_) {
          const size_t m = static_cast<size_t>(std::min<uint64_t>(k, c.left()));
          c.skip(m);
          consume(static_cast<uint32_t>(m));
          used += m;
          content_left_ -= m;
          if (content_left_ == 0) after_cd_field();
          continue;
        }
        // commit whatever the socket has now (not the whole frame), so the
        // sink's CRC / slot hand-off overlaps the rest arriving; a read past
        // the frame's end lands the following frames' payload contiguously
        uint64_t room = std::min<uint64_t>(k, w.cap);
        if (*delivered_ + room > cap_) room = std::min<uint64_t>(room, c.left());  // checked frame by frame
        const size_t m = c.read_spanning(w.ptr, static_cast<size_t>(room));
        if (*delivered_ + m > cap_) throw StorageError("ReadObject: server sent more than read_limit bytes", false);
        if (!rr_->first_byte_ns) rr_->first_byte_ns = now_ns();
        try {
          sink_.commit(m);
        } catch (const std::exception& e) {
          fail_sink(e.what());
        }
        *delivered_ += m;
        consume(static_cast<uint32_t>(m));
        used += m;
        content_left_ -= m;
        if (content_left_ == 0) after_cd_field();
        continue;
      }
      // token bytes (tags, lengths, fixed32, small fields): byte at a time
      uint8_t b = c.read_byte();
      consume(1);
      ++used;
      step(b);
    }
    return used;
  }

  void end() override {
    if (content_seen_ && !sink_failed_) {
      try {
        sink_.chunk_end(has_crc_, crc_);
      } catch (const std::exception& e) {
        fail_sink(e.what());
      }
      if (*call_ && sink_.deferred() && sink_.drain_wanted()) (*call_)->poke();
    }
  }

  bool sink_failed() const { return sink_failed_; }
  const std::string& sink_error() const { return sink_error_; }

 private:
  enum St {
    kTopTag, kTopLen, kCdLen, kCdTag, kContentLen, kContent, kCrc, kFieldBuf, kSkipVarint, kSkipFixed, kSkipLen,
    kSkipBytes
  };

  void fail_sink(const char* what) {
    if (!sink_failed_) {
      sink_failed_ = true;
      sink_error_ = what;
      if (*call_) (*call_)->handler_error(std::string("sink: ") + what);
    }
  }

  void consume(uint32_t k) {
    msg_left_ -= k;
    if (in_cd_) cd_left_ -= k;
  }

  bool varint_byte(uint8_t b, uint64_t* out) {
    vacc_ |= uint64_t(b & 0x7F) << vshift_;
    vshift_ += 7;
    if (b & 0x80) return false;
    *out = vacc_;
    vacc_ = 0;
    vshift_ = 0;
    return true;
  }

  void after_cd_field() {
    if (in_cd_ && cd_left_ == 0) in_cd_ = false;
    st_ = in_cd_ ? kCdTag : kTopTag;
  }

  void step(uint8_t b) {
    uint64_t v;
    switch (st_) {
      case kTopTag:
      case kCdTag:
        if (!varint_byte(b, &v)) return;
        field_ = static_cast<uint32_t>(v >> 3);
        wt_ = static_cast<uint32_t>(v & 7);
        if (st_ == kTopTag) {
          if (field_ == 1 && wt_ == pb::kLen) {
            st_ = kCdLen;
          } else if (wt_ == pb::kLen && (field_ == 2 || field_ == 3 || field_ == 4)) {
            st_ = kTopLen;
          } else {
            start_skip();
          }
        } else {  // inside checksummed_data
          if (field_ == 1 && wt_ == pb::kLen) st_ = kContentLen;
          else if (field_ == 2 && wt_ == pb::kI32) {
            st_ = kCrc;
            fixed_have_ = 0;
          } else start_skip();
        }
        return;
      case kCdLen:
        if (!varint_byte(b, &v)) return;
        in_cd_ = true;
        cd_left_ = v;
        st_ = v ? kCdTag : (in_cd_ = false, kTopTag);
        return;
      case kContentLen:
        if (!varint_byte(b, &v)) return;
        content_left_ = v;
        content_seen_ = true;
        if (!sink_failed_) {
          try {
            sink_.chunk_begin(static_cast<size_t>(v));
          } catch (const std::exception& e) {
            fail_sink(e.what());
          }
        }
        if (v) st_ = kContent;
        else after_cd_field();
        return;
      case kCrc:
        fixed_[fixed_have_++] = b;
        if (fixed_have_ == 4) {
          std::memcpy(&crc_, fixed_, 4);
          has_crc_ = true;
          after_cd_field();
        }
        return;
      case kTopLen:
        if (!varint_byte(b, &v)) return;
        fbuf_.clear();
        fbuf_len_ = v;
        st_ = kFieldBuf;
        if (v == 0) finish_field();
        return;
      case kSkipLen:
        if (!varint_byte(b, &v)) return;
        skip_left_ = v;
        if (v) st_ = kSkipBytes;
        else after_cd_field();
        return;
      case kFieldBuf:
        fbuf_.push_back(static_cast<char>(b));
        if (fbuf_.size() == fbuf_len_) finish_field();
        return;
      case kSkipVarint:
        if (!(b & 0x80)) after_cd_field();
        return;
      case kSkipFixed:
      case kSkipBytes:
        if (--skip_left_ == 0) after_cd_field();
        return;
      case kContent:
        return;
    }
  }

  void start_skip() {
    switch (wt_) {
      case pb::kVarint: st_ = kSkipVarint; break;
      case pb::kI64: st_ = kSkipFixed; skip_left_ = 8; break;
      case pb::kI32: st_ = kSkipFixed; skip_left_ = 4; break;
      case pb::kLen: st_ = kSkipLen; break;
      default: throw StorageError("ReadObjectResponse: unsupported wire type", false);
    }
  }

  void finish_field() {
    ObjectInfo info;
    bool changed = false;
    if (field_ == 2) {  // object_checksums
      std::string md5;
      if (v2::decode_checksums(fbuf_, &info.has_crc32c, &info.crc32c, &md5)) {
        info.md5 = md5;
        if (!full_read_) info.has_crc32c = false;
        rr_->info.has_crc32c = info.has_crc32c || rr_->info.has_crc32c;
        if (info.has_crc32c) rr_->info.crc32c = info.crc32c;
        changed = true;
      }
    } else if (field_ == 4) {  // metadata
      v2::Object o;
      if (v2::decode_object(fbuf_, &o)) {
        info.size = o.size;
        info.generation = o.generation;
        rr_->info.size = o.size;
        rr_->info.generation = o.generation;
        changed = true;
      }
    } else if (field_ == 3) {  // content_range
      v2::ContentRange cr;
      if (v2::decode_content_range(fbuf_, &cr) && cr.complete_length > 0) {
        info.size = cr.complete_length;
        rr_->info.size = cr.complete_length;
        changed = true;
      }
    }
    if (changed && !sink_failed_) {
      try {
        sink_.update_info(info);
      } catch (const std::exception& e) {
        fail_sink(e.what());
      }
    }
    st_ = kTopTag;
  }

  Sink& sink_;
  ReadResult* rr_;
  uint64_t* delivered_;
  bool full_read_;
  GrpcCall** call_;
  uint64_t cap_ = ~0ull;
  St st_ = kTopTag;
  uint64_t msg_left_ = 0, cd_left_ = 0, content_left_ = 0, skip_left_ = 0, fbuf_len_ = 0;
  bool in_cd_ = false, content_seen_ = false, has_crc_ = false;
  uint32_t crc_ = 0, field_ = 0, wt_ = 0;
  uint64_t vacc_ = 0;
  int vshift_ = 0;
  uint8_t fixed_[4];
  int fixed_have_ = 0;
  std::string fbuf_;
  bool sink_failed_ = false;
  std::string sink_error_;
};

class GrpcStorageClient : public StorageClient {
  std::string path_ = "cloudpath";

 public:
  explicit GrpcStorageClient(const ClientConfig& cfg) : StorageClient(cfg) {
    int n = std::max(1, cfg.grpc_conn_pool_size);
    conns_.resize(static_cast<size_t>(n));
    opt_.sock = cfg.sock;
    opt_.sock.alpn = "h2";  // gRPC over TLS negotiates HTTP/2 by ALPN
    // -read-timeout is per stream here: a socket timeout would kill the
    // shared reader thread of an idle multiplexed connection
    idle_ms_ = cfg.sock.io_timeout_ms;
    opt_.sock.io_timeout_ms = 0;
    opt_.cpus = cfg.reader_cpus.empty() ? cfg.cpus : cfg.reader_cpus;
    opt_.max_frame_size = cfg.h2_max_frame_size;
    opt_.initial_window = cfg.h2_window;
    opt_.span_max_frame = cfg.h2_span_max_frame;
    // DirectPath (reference main.go:106-117: GOOGLE_CLOUD_ENABLE_DIRECT_PATH_XDS
    // is set only around NewGRPCClient, with the google-c2p xDS resolver and
    // the RLS balancer linked in).  DirectPath needs the GCE metadata server,
    // an xDS bootstrap and ALTS; without them the library falls back to
    // CloudPath, and so does this client: the request is recorded, the
    // configured endpoint is used.
    const char* dp = std::getenv("GOOGLE_CLOUD_ENABLE_DIRECT_PATH_XDS");
    if (dp && std::string(dp) == "true") {
      const bool prod = cfg.endpoint.host == "storage.googleapis.com";
      path_ = prod ? "cloudpath (DirectPath requested: no xDS bootstrap / ALTS on this host)"
                   : "cloudpath (DirectPath requested: custom endpoint " + cfg.endpoint.host + ")";
    }
  }

  std::string transport_name() const override { return "grpc"; }
  std::string transport_path() const override { return path_; }

 protected:
  std::shared_ptr<H2ClientConn> conn() {
    size_t i = rr_.fetch_add(1) % conns_.size();
    std::lock_guard<std::mutex> lk(mu_);
    auto& c = conns_[i];
    if (!c || !c->usable()) {
      if (c) c->close();
      c = H2ClientConn::dial(cfg_.endpoint, opt_);
      ++stats_.dials;
    }
    return c;
  }

  HeaderList headers(const std::string& method, const std::string& bucket_res) {
    HeaderList h = {{":method", "POST"},
                    {":scheme", cfg_.endpoint.scheme == "https" ? "https" : "http"},
                    {":path", std::string(v2::kService) + method},
                    {":authority", cfg_.endpoint.host_header()},
                    {"content-type", "application/grpc"},
                    {"te", "trailers"},
                    {"grpc-accept-encoding", "identity"},
                    {"user-agent", "gcsb-native-grpc/0.1 (" + cfg_.user_agent + ")"}};
    if (!bucket_res.empty()) h.emplace_back("x-goog-request-params", "bucket=" + url_encode(bucket_res));
    if (cfg_.token) h.emplace_back("authorization", "Bearer " + cfg_.token->token());
    return h;
  }

  static std::string frame(const std::string& msg) {
    std::string f(5, '\0');
    put_be32(reinterpret_cast<uint8_t*>(&f[1]), static_cast<uint32_t>(msg.size()));
    f += msg;
    return f;
  }

  // Unary call returning the single response message.
  std::string unary(const std::string& method, const std::string& bucket_res, const std::string& req) {
    BufferingHandler h;
    auto call = std::make_shared<GrpcCall>(&h);
    auto c = conn();
    std::string f = frame(req);
    try {
      c->start_stream_with_body(call, headers(method, bucket_res), f);
      call->wait_ok(nullptr, idle_ms_, [c, call, this] { c->abandon_stream(*call, idle_ms_); });
    } catch (...) {
      c->end_stream(*call, true);
      throw;
    }
    c->end_stream(*call, false);
    if (h.messages().empty()) throw StorageError(method + ": no response message", true);
    return h.messages().front();
  }

  void read_attempt(const std::string& bucket, const std::string& object, Sink& sink, int64_t offset, int64_t limit,
                    bool first_attempt, ReadResult* rr, uint64_t* delivered) override {
    if (first_attempt) {
      ObjectInfo bi;
      bi.start_offset = offset;
      sink.begin(bi);
      rr->sink_begun = true;
      rr->info = bi;
    }
    // A whole-object read stays one: a resumed attempt (offset = delivered)
    // still feeds the CRC the sink has run from byte 0, so every attempt's
    // object_checksums apply -- the first attempt may have been cut before
    // its first message's checksums field arrived.
    const bool full = rr->info.start_offset == 0 && limit < 0;
    v2::ReadObjectRequest q;
    q.bucket = v2::bucket_resource(bucket);
    q.object = object;
    q.read_offset = offset;
    q.read_limit = limit > 0 ? limit : 0;
    q.generation = rr->pin_generation;
    GrpcCall* raw = nullptr;
    auto c = conn();
    ReadObjectHandler h(sink, rr, delivered, full, &raw, limit >= 0 ? *delivered + limit : ~0ull);
    auto call = std::make_shared<GrpcCall>(&h);
    raw = call.get();
    std::string f = frame(v2::encode_read_request(q));
    try {
      c->start_stream_with_body(call, headers("ReadObject", q.bucket), f);
      call->wait_ok(sink.deferred() ? &sink : nullptr, idle_ms_, [c, call, this] { c->abandon_stream(*call, idle_ms_); });
    } catch (...) {
      c->end_stream(*call, true);
      throw;
    }
    c->end_stream(*call, false);
    if (h.sink_failed()) throw StorageError("sink: " + h.sink_error(), false);
  }

  ObjectMeta from_v2(const v2::Object& o) {
    ObjectMeta m;
    m.name = o.name;
    m.bucket = v2::bucket_from_resource(o.bucket);
    m.size = o.size;
    m.generation = o.generation;
    m.metageneration = o.metageneration;
    m.has_crc32c = o.has_crc32c;
    m.crc32c = o.crc32c;
    m.md5 = o.md5;
    m.content_type = o.content_type;
    return m;
  }

  ObjectMeta stat_attempt(const std::string& bucket, const std::string& object) override {
    v2::GetObjectRequest q;
    q.bucket = v2::bucket_resource(bucket);
    q.object = object;
    std::string resp = unary("GetObject", q.bucket, v2::encode_get_request(q));
    v2::Object o;
    if (!v2::decode_object(resp, &o)) throw StorageError("GetObject: bad response", false);
    return from_v2(o);
  }

  ObjectMeta compose_attempt(const std::string& bucket, const std::string& dest,
                             const std::vector<std::string>& sources, const std::string& content_type) override {
    v2::ComposeObjectRequest q;
    q.destination.bucket = v2::bucket_resource(bucket);
    q.destination.name = dest;
    q.destination.content_type = content_type;
    q.sources = sources;
    std::string resp = unary("ComposeObject", q.destination.bucket, v2::encode_compose_request(q));
    v2::Object o;
    if (!v2::decode_object(resp, &o)) throw StorageError("ComposeObject: bad response", false);
    return from_v2(o);
  }

  void delete_attempt(const std::string& bucket, const std::string& object) override {
    v2::GetObjectRequest q;
    q.bucket = v2::bucket_resource(bucket);
    q.object = object;
    unary("DeleteObject", q.bucket, v2::encode_delete_request(q));
  }

  ListResult list_attempt(const std::string& bucket, const std::string& prefix, int page_size,
                          const std::string& page_token, const std::string& delimiter) override {
    v2::ListObjectsRequest q;
    q.parent = v2::bucket_resource(bucket);
    q.page_size = page_size;
    q.page_token = page_token;
    q.prefix = prefix;
    q.delimiter = delimiter;
    std::string resp = unary("ListObjects", q.parent, v2::encode_list_request(q));
    v2::ListObjectsResponse lr;
    if (!v2::decode_list_response(resp, &lr)) throw StorageError("ListObjects: bad response", false);
    ListResult r;
    for (auto& o : lr.objects) r.objects.push_back(from_v2(o));
    r.prefixes = lr.prefixes;
    r.next_page_token = lr.next_page_token;
    return r;
  }

  // Streams [from, total) of src as WriteObjectRequest messages on one call;
  // the last one carries the object's checksums, asked of the source only
  // then (a GPU source knows them once every slot was staged).
  ObjectMeta write_stream(const std::string& bucket_res, const std::string& upload_id, const std::string* spec,
                          ByteSource& src, uint64_t from, UploadPhases* ph = nullptr, int64_t t_base = 0) {
    const uint64_t total = src.size();
    const size_t kMsg = 2u << 20;  // ServiceConstants MAX_WRITE_CHUNK_BYTES [lib]
    BufferingHandler h;
    auto call = std::make_shared<GrpcCall>(&h);
    auto c = conn();
    // zero-copy send of the content (vmsplice + splice) when the source's
    // bytes stay put until the final response
    const bool splice = src.stable_until_done();
    constexpr size_t kMinSplice = 64 << 10;  // below this a copy is cheaper than 2 syscalls
    c->start_stream(call, headers("WriteObject", bucket_res), false);
    try {
      src.seek(from);
      uint64_t off = from;
      bool first = true;
      do {
        auto [p, k] = src.next(static_cast<size_t>(std::min<uint64_t>(kMsg, total - off)));
        bool last = off + k >= total;
        // per-message ChecksummedData CRC: precomputed on the GPU for HBM
        // sources (no host pass over the bytes), else SSE4.2 on the host
        uint32_t crc = 0;
        if (k && !src.range_crc32c(off, k, &crc)) crc = crc32c(p, k);
        const std::string object_checksums = last ? v2::encode_checksums(src.has_crc32c(), src.crc32c(), "")
                                                  : std::string();
        v2::WriteRequestParts parts = v2::encode_write_request(first ? upload_id : std::string(),
                                                               first ? spec : nullptr, static_cast<int64_t>(off), k,
                                                               k > 0, crc, last ? &object_checksums : nullptr, last);
        uint64_t mlen = parts.head.size() + k + parts.tail.size();
        uint8_t pre[5] = {0, 0, 0, 0, 0};
        put_be32(pre + 1, static_cast<uint32_t>(mlen));
        if (splice) {
          // the content by page reference: the source keeps it unchanged
          // until this upload's final response (ByteSource::stable_until_done)
          std::vector<SendPiece> pieces(4);
          pieces[0].p = pre;
          pieces[0].n = 5;
          pieces[1].p = reinterpret_cast<const uint8_t*>(parts.head.data());
          pieces[1].n = parts.head.size();
          pieces[2].p = p;
          pieces[2].n = k;
          pieces[2].splice = k >= kMinSplice;
          pieces[3].p = reinterpret_cast<const uint8_t*>(parts.tail.data());
          pieces[3].n = parts.tail.size();
          c->send_data_pieces(*call, pieces, last);
        } else {
          iovec iov[4] = {{pre, 5},
                          {parts.head.data(), parts.head.size()},
                          {const_cast<uint8_t*>(p), k},
                          {parts.tail.data(), parts.tail.size()}};
          c->send_data_iov(*call, iov, 4, last);
        }
        if (first && ph) ph->first_send_ns = now_ns() - t_base;
        if (last && ph) ph->last_send_ns = now_ns() - t_base;
        off += k;
        first = false;
        if (last) break;
        if (k == 0) throw StorageError("upload source ended early", false);
      } while (true);
      // The final response gets its own, longer idle bound (10 x
      // -read-timeout): a server may take longer than
      // -read-timeout to finalize a large object.  Running out of it is NOT
      // retryable: the whole upload sent again could duplicate a generation
      // the first one committed.
      const int fin_ms = idle_ms_ > 0 ? 10 * idle_ms_ : 0;
      try {
        call->wait_ok(nullptr, fin_ms, [c, call, fin_ms] { c->abandon_stream(*call, fin_ms); });
      } catch (const StorageError& e) {
        if (fin_ms > 0 && std::strncmp(e.what(), "read timeout", 12) == 0)
          throw StorageError("WriteObject: no final response within " + std::to_string(fin_ms) +
                                 " ms of the last byte (not retried: the upload may have committed)",
                             false);
        throw;
      }
    } catch (...) {
      c->end_stream(*call, true);
      throw;
    }
    c->end_stream(*call, false);
    if (ph) ph->response_ns = now_ns() - t_base;
    if (h.messages().empty()) throw StorageError("WriteObject: no response", true);
    v2::WriteStatus st;
    if (!v2::decode_write_status(h.messages().front(), &st) || !st.has_resource)
      throw StorageError("WriteObject: response without resource", false);
    return from_v2(st.resource);
  }

  ObjectMeta write_impl(const std::string& bucket, const std::string& object, ByteSource& src,
                        const WriteOptions& opt) override {
    const std::string bres = v2::bucket_resource(bucket);
    // this upload's phases, published however it returns
    struct Phases {
      GrpcStorageClient* self;
      UploadPhases ph;
      const int64_t t0 = now_ns();
      ~Phases() { self->set_last_upload(ph); }
    } up{this, {}};
    v2::WriteObjectSpec spec;
    spec.resource.name = object;
    spec.resource.bucket = bres;
    spec.resource.content_type = opt.content_type;
    spec.object_size = static_cast<int64_t>(src.size());
    if (!opt.resumable) {
      const std::string sp = v2::encode_write_spec(spec);
      return with_retry([&] { return write_stream(bres, "", &sp, src, 0, &up.ph, up.t0); });
    }
    std::string upload_id;
    {
      // the object's checksums up front only when the source already has
      // them; else they ride in the last WriteObjectRequest (finish_write)
      const std::string checksums =
          src.crc32c_ready() ? v2::encode_checksums(src.has_crc32c(), src.crc32c(), "") : std::string();
      std::string resp = with_retry([&] {
        return unary("StartResumableWrite", bres,
                     v2::encode_start_resumable(spec, checksums.empty() ? nullptr : &checksums));
      });
      if (!v2::decode_upload_id(resp, &upload_id) || upload_id.empty())
        throw StorageError("StartResumableWrite: no upload_id", false);
      up.ph.start_rpc_ns = now_ns() - up.t0;
    }
    Backoff bo(cfg_.retry);
    int64_t t0 = now_ns();
    uint64_t from = 0;
    for (int attempt = 1;; ++attempt) {
      try {
        return write_stream(bres, upload_id, nullptr, src, from, &up.ph, up.t0);
      } catch (const StorageError& e) {
        if (!should_retry(cfg_.retry, e, attempt, t0)) throw;
        ++stats_.retries;
        sleep_seconds(bo.pause());
        try {
          std::string resp = unary("QueryWriteStatus", bres, v2::encode_upload_id(upload_id));
          v2::WriteStatus st;
          v2::decode_write_status(resp, &st);
          if (st.has_resource) return from_v2(st.resource);
          from = static_cast<uint64_t>(st.persisted_size);
        } catch (const StorageError&) {
        }
      }
    }
  }

 private:
  H2ClientOptions opt_;
  int idle_ms_ = 0;
  std::mutex mu_;
  std::vector<std::shared_ptr<H2ClientConn>> conns_;
  std::atomic<uint64_t> rr_{0};
};

}  // namespace

std::unique_ptr<StorageClient> make_grpc_client(const ClientConfig& cfg) {
  return std::make_unique<GrpcStorageClient>(cfg);
}

}  // namespace gcsb
