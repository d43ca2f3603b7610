#include "h2/h2_client.h"

#include <sys/socket.h>
#include <sys/uio.h>

#include <chrono>
#include <cstring>
#include <thread>

#include "core/affinity.h"
#include "core/util.h"

namespace gcsb {

namespace {
std::atomic<uint64_t> g_frames{0}, g_data_frames{0}, g_header_blocks{0}, g_data_bytes{0}, g_wait_ns{0},
    g_data_ns{0}, g_headers_ns{0}, g_other_ns{0}, g_long_waits{0}, g_long_wait_ns{0}, g_readers{0},
    g_spanned_frames{0}, g_span_reads{0}, g_span_spills{0};
constexpr int kMaxSpanFrames = 64;  // frames one read_spanning plan covers (1 MiB of 16 KiB frames)
constexpr int64_t kLongWaitNs = 5000000;
}  // namespace

H2ReaderStats h2_reader_stats() {
  H2ReaderStats s;
  s.frames = g_frames.load();
  s.data_frames = g_data_frames.load();
  s.header_blocks = g_header_blocks.load();
  s.data_bytes = g_data_bytes.load();
  s.header_wait_ns = g_wait_ns.load();
  s.data_ns = g_data_ns.load();
  s.headers_ns = g_headers_ns.load();
  s.other_ns = g_other_ns.load();
  s.long_waits = g_long_waits.load();
  s.long_wait_ns = g_long_wait_ns.load();
  s.readers_alive = g_readers.load();
  s.spanned_frames = g_spanned_frames.load();
  s.span_reads = g_span_reads.load();
  s.span_spills = g_span_spills.load();
  return s;
}

// --- H2DataCursor ------------------------------------------------------------

void H2DataCursor::read_exact(void* dst, size_t n) {
  if (n > left_) throw StorageError("http2: read past the end of a DATA frame", false);
  bc_->read_exact(dst, n);
  left_ -= static_cast<uint32_t>(n);
}

uint8_t H2DataCursor::read_byte() {
  if (left_ == 0) throw StorageError("http2: read past the end of a DATA frame", false);
  --left_;
  return bc_->read_byte();
}

void H2DataCursor::skip(size_t n) {
  if (n > left_) throw StorageError("http2: skip past the end of a DATA frame", false);
  bc_->skip(n);
  left_ -= static_cast<uint32_t>(n);
}

size_t H2DataCursor::read_some(void* dst, size_t n) {
  n = std::min<size_t>(n, left_);
  if (n == 0) throw StorageError("http2: read past the end of a DATA frame", false);
  const size_t m = bc_->read_some(dst, n);
  if (m == 0) throw StorageError("connection closed inside a DATA frame", true);
  left_ -= static_cast<uint32_t>(m);
  return m;
}

void H2DataCursor::spill(const struct iovec* iov, int cnt, size_t i, size_t off, size_t n) {
  g_span_spills.fetch_add(1, std::memory_order_relaxed);
  std::vector<uint8_t> v;
  v.reserve(n);
  for (; n > 0 && static_cast<int>(i) < cnt; ++i, off = 0) {
    const size_t k = std::min(n, iov[i].iov_len - off);
    const auto* p = static_cast<const uint8_t*>(iov[i].iov_base) + off;
    v.insert(v.end(), p, p + k);
    n -= k;
  }
  bc_->unread(v.data(), v.size());
}

size_t H2DataCursor::read_spanning(uint8_t* dst, size_t want) {
  if (want <= left_ || !can_span_ || end_ || left_ == 0 || bc_->buffered() > 0)
    return read_some(dst, want);
  // the plan: [rest of this frame -> dst] then per frame [header -> hdr[j]]
  // [payload -> right after the previous payload in dst]
  uint8_t hdr[kMaxSpanFrames][9];
  iovec iov[2 * kMaxSpanFrames + 1];
  uint32_t plen[kMaxSpanFrames];
  int cnt = 0, nf = 0;
  iov[cnt++] = {dst, left_};
  size_t placed = left_;
  while (placed < want && nf < kMaxSpanFrames) {
    iov[cnt++] = {hdr[nf], 9};
    plen[nf] = static_cast<uint32_t>(std::min<size_t>(max_frame_, want - placed));
    iov[cnt++] = {dst + placed, plen[nf]};
    placed += plen[nf];
    ++nf;
  }
  g_span_reads.fetch_add(1, std::memory_order_relaxed);
  const size_t r = bc_->recv_scatter(iov, cnt);
  if (r <= left_) {
    left_ -= static_cast<uint32_t>(r);
    return r;
  }
  size_t got = left_, rem = r - left_;
  left_ = 0;
  for (int j = 0; j < nf; ++j) {
    const size_t hi = 1 + 2 * static_cast<size_t>(j);  // iov index of frame j's header
    if (rem < 9) {  // the header is still on its way: the reader loop reads it
      if (rem) spill(iov, cnt, hi, 0, rem);
      return got;
    }
    const uint8_t* b = hdr[j];
    const uint32_t len = (uint32_t(b[0]) << 16) | (uint32_t(b[1]) << 8) | b[2];
    const uint32_t sid = be32(b + 5) & 0x7FFFFFFF;
    if (b[3] != h2::kData || sid != stream_ || b[4] != 0 || len > max_frame_) {
      // not a plain DATA frame of this stream: the reader loop dispatches it
      spill(iov, cnt, hi, 0, rem);
      return got;
    }
    rem -= 9;
    ++spanned_frames_;
    spanned_wire_ += len;
    const size_t take = std::min<size_t>({rem, plen[j], len});
    got += take;
    rem -= take;
    left_ = len - static_cast<uint32_t>(take);
    if (rem == 0) return got;  // what is left of frame j is still on the socket
    if (take < plen[j]) {
      // frame j was shorter than planned: what follows it is not where the
      // plan put it
      spill(iov, cnt, hi + 1, take, rem);
      return got;
    }
  }
  return got;  // every planned frame came whole (bytes past the plan are buffered)
}

std::shared_ptr<H2ClientConn> H2ClientConn::dial(const Endpoint& ep, const H2ClientOptions& opt) {
  std::shared_ptr<H2ClientConn> c(new H2ClientConn(ep, opt));
  auto conn = Conn::dial(ep, opt.sock);
  if (conn->tls() && conn->alpn() != "h2")
    throw StorageError("TLS peer " + ep.host + " did not negotiate h2 (ALPN '" + conn->alpn() + "')", false);
  c->bc_ = std::make_unique<BufferedConn>(std::move(conn));
  c->w_ = std::make_unique<H2Writer>(c->bc_->conn());
  c->dec_ = HpackDecoder(opt.header_table_size);
  // connection preface + our SETTINGS + open the connection window wide
  c->bc_->conn().write_all(h2::kPreface, 24);
  std::vector<std::pair<uint16_t, uint32_t>> settings = {{h2::kSettingsEnablePush, 0},
                                                         {h2::kSettingsInitialWindowSize, opt.initial_window},
                                                         {h2::kSettingsHeaderTableSize, opt.header_table_size}};
  // max_frame_size 0: not advertised, the peer keeps the RFC default (16 KiB)
  if (opt.max_frame_size) settings.push_back({h2::kSettingsMaxFrameSize, opt.max_frame_size});
  c->w_->write_settings(encode_settings(settings));
  // the connection window opens to the stream window's size
  if (opt.initial_window > h2::kDefaultWindow) c->w_->write_window_update(0, opt.initial_window - h2::kDefaultWindow);
  c->conn_recv_.set_threshold(RecvWindow::threshold_for(std::max(opt.initial_window, h2::kDefaultWindow), 64 << 20));
  c->reader_ = std::thread([raw = c.get()] {
    pin_current_thread(raw->opt_.cpus);
    name_current_thread("gcsb-h2-reader");
    raw->reader_loop();
  });
  return c;
}

H2ClientConn::~H2ClientConn() { close(); }

void H2ClientConn::close() {
  if (!dead_.exchange(true) && w_) {  // w_ is null if dial() failed before the preface
    try {
      w_->write_goaway(0, h2::kErrNoError, "");
    } catch (...) {
    }
  }
  if (bc_) ::shutdown(bc_->conn().fd(), SHUT_RDWR);
  if (w_) w_->kill();
  // two threads may close one connection (a timed-out stream's watchdog and
  // the pool replacing the dead connection): one of them joins the reader
  std::lock_guard<std::mutex> lk(close_mu_);
  if (reader_.joinable()) {
    if (reader_.get_id() == std::this_thread::get_id())
      reader_.detach();
    else
      reader_.join();
  }
}

size_t H2ClientConn::active_streams() {
  std::lock_guard<std::mutex> lk(mu_);
  return streams_.size();
}

std::shared_ptr<H2ClientStream> H2ClientConn::acquire(uint32_t id) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = streams_.find(id);
  if (it == streams_.end()) return nullptr;
  it->second->busy_.fetch_add(1, std::memory_order_relaxed);
  return it->second;
}

bool H2ClientConn::cancel_stream(H2ClientStream& s, int wait_ms) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (s.id_ == 0 || s.cancelled_) return true;
    streams_.erase(s.id_);
    s.cancelled_ = true;
  }
  // no dispatch into s can start now; wait out one that already has
  const int64_t deadline = now_ns() + static_cast<int64_t>(std::max(wait_ms, 1)) * 1000000;
  while (s.busy_.load(std::memory_order_acquire) > 0) {
    if (now_ns() > deadline) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  w_->unregister_stream(s.id_);
  if (usable()) {
    try {
      w_->write_rst(s.id_, h2::kErrCancel);
    } catch (...) {
    }
  }
  return true;
}

void H2ClientConn::abandon_stream(H2ClientStream& s, int idle_ms) {
  const int64_t quiet_ns = now_ns() - last_frame_ns_.load(std::memory_order_relaxed);
  if (usable() && quiet_ns < static_cast<int64_t>(idle_ms) * 1000000 && cancel_stream(s, idle_ms)) return;
  close();
}

void H2ClientConn::start_stream(const std::shared_ptr<H2ClientStream>& s, const HeaderList& headers,
                                bool end_stream) {
  std::string block;
  enc_.encode(headers, &block);
  std::lock_guard<std::mutex> olk(open_mu_);  // stream ids must hit the wire in order
  if (!usable()) throw StorageError("http2 connection unusable: " + dead_reason(), true);
  if (next_id_ > 0x7FFFFFF0) {
    goaway_ = true;
    throw StorageError("http2 stream ids exhausted", true);
  }
  s->id_ = next_id_;
  s->conn_frames_ = &frames_;
  s->recv_window_.set_threshold(RecvWindow::threshold_for(opt_.initial_window, 16 << 20));
  next_id_ += 2;
  {
    std::lock_guard<std::mutex> lk(mu_);
    streams_[s->id_] = s;
  }
  w_->register_stream(s->id_);
  try {
    w_->write_headers(s->id_, block, end_stream);
  } catch (const StorageError& e) {
    dead_ = true;
    throw;
  }
}

void H2ClientConn::start_stream_with_body(const std::shared_ptr<H2ClientStream>& s, const HeaderList& headers,
                                          const std::string& body) {
  std::string block;
  enc_.encode(headers, &block);
  {
    std::lock_guard<std::mutex> olk(open_mu_);
    if (!usable()) throw StorageError("http2 connection unusable: " + dead_reason(), true);
    if (next_id_ > 0x7FFFFFF0) {
      goaway_ = true;
      throw StorageError("http2 stream ids exhausted", true);
    }
    s->id_ = next_id_;
    s->conn_frames_ = &frames_;
    s->recv_window_.set_threshold(RecvWindow::threshold_for(opt_.initial_window, 16 << 20));
    next_id_ += 2;
    {
      std::lock_guard<std::mutex> lk(mu_);
      streams_[s->id_] = s;
    }
    w_->register_stream(s->id_);
    try {
      if (w_->write_headers_and_data(s->id_, block, reinterpret_cast<const uint8_t*>(body.data()), body.size()))
        return;
      w_->write_headers(s->id_, block, false);
    } catch (const StorageError& e) {
      dead_ = true;
      throw;
    }
  }
  send_data(*s, reinterpret_cast<const uint8_t*>(body.data()), body.size(), true);
}

void H2ClientConn::send_data(H2ClientStream& s, const uint8_t* p, size_t n, bool end_stream) {
  iovec iov{const_cast<uint8_t*>(p), n};
  send_data_iov(s, &iov, 1, end_stream);
}

void H2ClientConn::send_data_iov(H2ClientStream& s, struct iovec* iov, int cnt, bool end_stream) {
  size_t total = 0;
  for (int i = 0; i < cnt; ++i) total += iov[i].iov_len;
  if (total == 0) {
    if (end_stream) w_->write_frame(h2::kData, h2::kFlagEndStream, s.id_, nullptr, 0);
    return;
  }
  int idx = 0;
  size_t off = 0;  // offset inside iov[idx]
  size_t left = total;
  std::vector<iovec> piece;
  while (left > 0) {
    size_t n = w_->reserve(s.id_, left);
    if (n == 0) throw StorageError("http2 stream closed while sending: " + dead_reason(), true);
    piece.clear();
    size_t need = n;
    while (need > 0) {
      size_t k = std::min(need, iov[idx].iov_len - off);
      piece.push_back({static_cast<uint8_t*>(iov[idx].iov_base) + off, k});
      need -= k;
      off += k;
      if (off == iov[idx].iov_len) {
        ++idx;
        off = 0;
      }
    }
    left -= n;
    w_->write_frame_iov(h2::kData, (left == 0 && end_stream) ? h2::kFlagEndStream : 0, s.id_, piece.data(),
                        static_cast<int>(piece.size()), n);
  }
}

void H2ClientConn::send_data_pieces(H2ClientStream& s, const std::vector<SendPiece>& pieces, bool end_stream) {
  size_t total = 0;
  for (const SendPiece& p : pieces) total += p.n;
  if (total == 0) {
    if (end_stream) w_->write_frame(h2::kData, h2::kFlagEndStream, s.id_, nullptr, 0);
    return;
  }
  size_t idx = 0, off = 0, left = total;
  std::vector<SendPiece> frame;
  while (left > 0) {
    size_t n = w_->reserve(s.id_, left);
    if (n == 0) throw StorageError("http2 stream closed while sending: " + dead_reason(), true);
    frame.clear();
    size_t need = n;
    while (need > 0) {
      const SendPiece& src = pieces[idx];
      SendPiece q = src;
      const size_t k = std::min(need, src.n - off);
      q.p = src.p ? src.p + off : nullptr;
      q.foff = src.foff + off;
      q.n = k;
      frame.push_back(q);
      need -= k;
      off += k;
      if (off == src.n) {
        ++idx;
        off = 0;
      }
    }
    left -= n;
    w_->write_frame_pieces(h2::kData, (left == 0 && end_stream) ? h2::kFlagEndStream : 0, s.id_, frame, n);
  }
}

void H2ClientConn::end_stream(H2ClientStream& s, bool reset) {
  if (s.id_ == 0 || s.cancelled_) return;
  {
    std::lock_guard<std::mutex> lk(mu_);
    streams_.erase(s.id_);
  }
  w_->unregister_stream(s.id_);
  if (reset && usable()) {
    try {
      w_->write_rst(s.id_, h2::kErrCancel);
    } catch (...) {
    }
  }
}

void H2ClientConn::fail_all(const std::string& msg) {
  {
    std::lock_guard<std::mutex> lk(reason_mu_);
    if (dead_reason_.empty()) dead_reason_ = msg;
  }
  dead_ = true;
  w_->kill();
  std::map<uint32_t, std::shared_ptr<H2ClientStream>> s;
  {
    std::lock_guard<std::mutex> lk(mu_);
    s.swap(streams_);
  }
  for (auto& kv : s) kv.second->on_conn_error(msg);
}

void H2ClientConn::reader_loop() {
  std::string hblock;
  uint32_t hstream = 0;
  bool hend_stream = false;
  g_readers.fetch_add(1, std::memory_order_relaxed);
  struct Alive {
    ~Alive() { g_readers.fetch_sub(1, std::memory_order_relaxed); }
  } alive;
  try {
    for (;;) {
      const int64_t t_wait = now_ns();
      FrameHeader fh = read_frame_header(*bc_);
      const int64_t t_frame = now_ns();
      last_frame_ns_.store(t_frame, std::memory_order_relaxed);
      frames_.fetch_add(1, std::memory_order_relaxed);
      g_wait_ns.fetch_add(static_cast<uint64_t>(t_frame - t_wait), std::memory_order_relaxed);
      if (t_frame - t_wait > kLongWaitNs) {
        g_long_waits.fetch_add(1, std::memory_order_relaxed);
        g_long_wait_ns.fetch_add(static_cast<uint64_t>(t_frame - t_wait), std::memory_order_relaxed);
      }
      g_frames.fetch_add(1, std::memory_order_relaxed);
      struct Account {  // time of this frame's handling, by type
        uint8_t type;
        int64_t t0;
        ~Account() {
          const uint64_t d = static_cast<uint64_t>(now_ns() - t0);
          (type == h2::kData ? g_data_ns
                             : (type == h2::kHeaders || type == h2::kContinuation) ? g_headers_ns : g_other_ns)
              .fetch_add(d, std::memory_order_relaxed);
        }
      } account{fh.type, t_frame};
      if (fh.length > accept_max_frame()) throw StorageError("http2: frame exceeds max_frame_size", true);
      switch (fh.type) {
        case h2::kData: {
          uint32_t n = fh.length;
          uint8_t pad = 0;
          if (fh.flags & h2::kFlagPadded) {
            // RFC 7540 6.1: padding >= payload length is a PROTOCOL_ERROR
            if (n < 1) throw StorageError("http2: padded DATA frame without a pad length", false);
            pad = bc_->read_byte();
            if (static_cast<uint32_t>(pad) + 1 > n) throw StorageError("http2: DATA padding exceeds frame", false);
            n -= 1 + pad;
          }
          auto s = acquire(fh.stream);
          bool end = fh.flags & h2::kFlagEndStream;
          const uint32_t amax = accept_max_frame();
          H2DataCursor cur(*bc_, fh.stream, n, end,
                           pad == 0 && opt_.span_max_frame > 0 && amax <= opt_.span_max_frame, amax);
          if (s) {
            s->progress_.fetch_add(1, std::memory_order_relaxed);
            s->on_data(cur);
            s->progress_.fetch_add(1, std::memory_order_relaxed);
            release(*s);
          }
          if (cur.left()) bc_->skip(cur.left());  // an unknown stream, or one that left bytes
          if (pad) bc_->skip(pad);
          end = cur.end_stream();
          const uint64_t extra = cur.spanned_frames_;
          const uint64_t wire = fh.length + cur.spanned_wire_;
          g_data_frames.fetch_add(1 + extra, std::memory_order_relaxed);
          g_data_bytes.fetch_add(wire - (fh.length - n), std::memory_order_relaxed);
          if (extra) {
            g_frames.fetch_add(extra, std::memory_order_relaxed);
            g_spanned_frames.fetch_add(extra, std::memory_order_relaxed);
            frames_.fetch_add(extra, std::memory_order_relaxed);
            last_frame_ns_.store(now_ns(), std::memory_order_relaxed);
          }
          // replenish flow-control credit (connection + stream)
          if (uint32_t inc = conn_recv_.consume(static_cast<uint32_t>(wire))) w_->write_window_update(0, inc);
          if (s && !end)
            if (uint32_t inc = s->recv_window_.consume(static_cast<uint32_t>(wire)))
              w_->write_window_update(fh.stream, inc);
          break;
        }
        case h2::kHeaders:
        case h2::kContinuation: {
          std::string frag(fh.length, '\0');
          if (fh.length) bc_->read_exact(&frag[0], fh.length);
          size_t b = 0, e = frag.size();
          if (fh.type == h2::kHeaders) {
            hstream = fh.stream;
            hend_stream = fh.flags & h2::kFlagEndStream;
            hblock.clear();
            if (fh.flags & h2::kFlagPadded) {
              if (frag.empty()) throw StorageError("http2: padded HEADERS frame without a pad length", false);
              uint8_t pad = static_cast<uint8_t>(frag[0]);
              b = 1;
              if (static_cast<size_t>(pad) + 1 > e) throw StorageError("http2: HEADERS padding exceeds frame", false);
              e -= pad;
            }
            if (fh.flags & h2::kFlagPriority) b += 5;
            if (b > e) throw StorageError("http2: HEADERS frame too short", false);
          }
          hblock.append(frag, b, e - b);
          if (fh.flags & h2::kFlagEndHeaders) {
            g_header_blocks.fetch_add(1, std::memory_order_relaxed);
            HeaderList hl;
            dec_.decode(reinterpret_cast<const uint8_t*>(hblock.data()), hblock.size(), &hl);
            if (auto s = acquire(hstream)) {
              s->progress_.fetch_add(1, std::memory_order_relaxed);
              s->on_headers(hl, hend_stream);
              release(*s);
            }
          }
          break;
        }
        case h2::kRstStream: {
          if (fh.length != 4) throw StorageError("http2: RST_STREAM length != 4", false);
          uint8_t v[4];
          bc_->read_exact(v, 4);
          if (auto s = acquire(fh.stream)) {
            s->on_reset(be32(v));
            release(*s);
          }
          break;
        }
        case h2::kSettings: {
          std::string p(fh.length, '\0');
          if (fh.length) bc_->read_exact(&p[0], fh.length);
          if (!(fh.flags & h2::kFlagAck)) {
            uint32_t old = peer_.initial_window_size;
            if (!apply_settings_payload(reinterpret_cast<const uint8_t*>(p.data()), p.size(), &peer_))
              throw StorageError("http2: bad SETTINGS", true);
            w_->on_peer_settings(peer_, old);
            w_->write_settings_ack();
          }
          break;
        }
        case h2::kPing: {
          if (fh.length != 8) throw StorageError("http2: PING length != 8", false);
          uint8_t op[8];
          bc_->read_exact(op, 8);
          if (!(fh.flags & h2::kFlagAck)) w_->write_ping_ack(op);
          break;
        }
        case h2::kGoaway: {
          if (fh.length < 8) throw StorageError("http2: GOAWAY shorter than 8 bytes", false);
          std::string p(fh.length, '\0');
          bc_->read_exact(&p[0], fh.length);
          goaway_last_ = be32(reinterpret_cast<const uint8_t*>(p.data())) & 0x7FFFFFFF;
          goaway_ = true;
          std::vector<std::shared_ptr<H2ClientStream>> doomed;
          {
            std::lock_guard<std::mutex> lk(mu_);
            for (auto it = streams_.begin(); it != streams_.end();) {
              if (it->first > goaway_last_) {
                doomed.push_back(it->second);
                it = streams_.erase(it);
              } else {
                ++it;
              }
            }
          }
          for (auto& s : doomed) s->on_conn_error("GOAWAY");
          break;
        }
        case h2::kWindowUpdate: {
          if (fh.length != 4) throw StorageError("http2: WINDOW_UPDATE length != 4", false);
          uint8_t v[4];
          bc_->read_exact(v, 4);
          w_->on_window_update(fh.stream, be32(v) & 0x7FFFFFFF);
          break;
        }
        default:
          bc_->skip(fh.length);  // PRIORITY, unknown extension frames
      }
    }
  } catch (const std::exception& e) {
    fail_all(e.what());
  }
}

}  // namespace gcsb
