#include "h2/h2.h"

#include <sys/uio.h>

#include <chrono>
#include <cstring>
#include <stdexcept>

#include "core/util.h"

namespace gcsb {

const char h2::kPreface[25] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";

void encode_frame_header(uint8_t o[9], uint32_t len, uint8_t type, uint8_t flags, uint32_t stream) {
  o[0] = static_cast<uint8_t>(len >> 16);
  o[1] = static_cast<uint8_t>(len >> 8);
  o[2] = static_cast<uint8_t>(len);
  o[3] = type;
  o[4] = flags;
  o[5] = static_cast<uint8_t>((stream >> 24) & 0x7F);
  o[6] = static_cast<uint8_t>(stream >> 16);
  o[7] = static_cast<uint8_t>(stream >> 8);
  o[8] = static_cast<uint8_t>(stream);
}

FrameHeader read_frame_header(BufferedConn& bc) {
  uint8_t b[9];
  bc.read_exact(b, 9);
  FrameHeader h;
  h.length = (uint32_t(b[0]) << 16) | (uint32_t(b[1]) << 8) | b[2];
  h.type = b[3];
  h.flags = b[4];
  h.stream = be32(b + 5) & 0x7FFFFFFF;
  return h;
}

std::string encode_settings(const std::vector<std::pair<uint16_t, uint32_t>>& kv) {
  std::string s;
  for (const auto& e : kv) {
    s.push_back(static_cast<char>(e.first >> 8));
    s.push_back(static_cast<char>(e.first));
    uint8_t v[4];
    put_be32(v, e.second);
    s.append(reinterpret_cast<char*>(v), 4);
  }
  return s;
}

bool apply_settings_payload(const uint8_t* p, size_t n, H2Settings* s) {
  if (n % 6) return false;
  for (size_t i = 0; i < n; i += 6) {
    uint16_t id = static_cast<uint16_t>((p[i] << 8) | p[i + 1]);
    uint32_t v = be32(p + i + 2);
    switch (id) {
      case h2::kSettingsHeaderTableSize: s->header_table_size = v; break;
      case h2::kSettingsEnablePush: s->enable_push = v; break;
      case h2::kSettingsMaxConcurrentStreams: s->max_concurrent_streams = v; break;
      case h2::kSettingsInitialWindowSize:
        if (v > static_cast<uint32_t>(h2::kMaxWindow)) return false;
        s->initial_window_size = v;
        break;
      case h2::kSettingsMaxFrameSize:
        if (v < h2::kDefaultMaxFrame || v > h2::kMaxFrameLimit) return false;
        s->max_frame_size = v;
        break;
      case h2::kSettingsMaxHeaderListSize: s->max_header_list_size = v; break;
      default: break;  // unknown settings are ignored
    }
  }
  return true;
}

namespace {
thread_local int64_t t_last_wait_ns = 0;
}

void FifoLock::lock() {
  std::unique_lock<std::mutex> lk(mu_);
  if (!held_) {
    held_ = true;
    t_last_wait_ns = 0;
    return;
  }
  const int64_t t0 = now_ns();
  Waiter w;
  q_.push_back(&w);
  w.cv.wait(lk, [&] { return w.granted; });  // ownership handed over by unlock()
  t_last_wait_ns = now_ns() - t0;
}

bool FifoLock::try_lock() {
  std::lock_guard<std::mutex> lk(mu_);
  if (held_) return false;
  held_ = true;
  t_last_wait_ns = 0;
  return true;
}

void FifoLock::unlock() {
  std::lock_guard<std::mutex> lk(mu_);
  if (q_.empty()) {
    held_ = false;
    return;
  }
  Waiter* w = q_.front();
  q_.pop_front();
  w->granted = true;  // held_ stays set: the lock passes to the oldest waiter
  w->cv.notify_one();  // under mu_: w lives on the waiter's stack until it sees granted
}

int64_t FifoLock::last_wait_ns() { return t_last_wait_ns; }

void note_send(H2SendStats& st, uint64_t wait_ns) {
  st.data_frames.fetch_add(1, std::memory_order_relaxed);
  st.queue_wait_ns.fetch_add(wait_ns, std::memory_order_relaxed);
  uint64_t m = st.queue_wait_max_ns.load(std::memory_order_relaxed);
  while (wait_ns > m && !st.queue_wait_max_ns.compare_exchange_weak(m, wait_ns, std::memory_order_relaxed)) {
  }
}

void H2Writer::note_data_frame() {
  const uint64_t w = static_cast<uint64_t>(FifoLock::last_wait_ns());
  note_send(sstats_, w);
  if (sink_) note_send(*sink_, w);
}

void H2Writer::release() {
  for (;;) {
    std::string pend;
    {
      std::lock_guard<std::mutex> lk(ctl_mu_);
      if (ctl_pending_.empty()) {
        wmu_.unlock();  // under ctl_mu_: a control frame queued after this check finds wmu_ free
        return;
      }
      pend.swap(ctl_pending_);
    }
    try {
      conn_.write_all(pend.data(), pend.size());
    } catch (...) {
      // the connection is gone; its reader fails every stream
    }
  }
}

void H2Writer::write_control(uint8_t type, uint8_t flags, uint32_t stream, const void* p, size_t n) {
  std::string f(9 + n, '\0');
  encode_frame_header(reinterpret_cast<uint8_t*>(&f[0]), static_cast<uint32_t>(n), type, flags, stream);
  if (n) std::memcpy(&f[9], p, n);
  {
    std::lock_guard<std::mutex> lk(ctl_mu_);
    ctl_pending_ += f;
    // a holder checks ctl_pending_ under ctl_mu_ before it unlocks: either it
    // sees this frame, or wmu_ is free now and this thread sends it
    if (!wmu_.try_lock()) return;
  }
  release();
}

void H2Writer::write_frame(uint8_t type, uint8_t flags, uint32_t stream, const void* p, size_t n) {
  uint8_t hdr[9];
  encode_frame_header(hdr, static_cast<uint32_t>(n), type, flags, stream);
  iovec iov[2] = {{hdr, 9}, {const_cast<void*>(p), n}};
  WriteLock lk(*this);
  if (type == h2::kData) note_data_frame();
  conn_.writev_all(iov, n ? 2 : 1);
}

void H2Writer::write_frame_iov(uint8_t type, uint8_t flags, uint32_t stream, struct iovec* payload, int cnt,
                               size_t total) {
  uint8_t hdr[9];
  encode_frame_header(hdr, static_cast<uint32_t>(total), type, flags, stream);
  std::vector<iovec> iov(static_cast<size_t>(cnt) + 1);
  iov[0] = {hdr, 9};
  for (int i = 0; i < cnt; ++i) iov[static_cast<size_t>(i) + 1] = payload[i];
  WriteLock lk(*this);
  if (type == h2::kData) note_data_frame();
  conn_.writev_all(iov.data(), cnt + 1);
}

void H2Writer::write_frame_pieces(uint8_t type, uint8_t flags, uint32_t stream, const std::vector<SendPiece>& pieces,
                                  size_t total, const std::string* lead_headers, const std::string* trailers) {
  uint8_t hdr[9], lh[9], th[9];
  encode_frame_header(hdr, static_cast<uint32_t>(total), type, flags, stream);
  std::vector<iovec> iov;
  iov.reserve(pieces.size() + 5);
  if (lead_headers) {
    encode_frame_header(lh, static_cast<uint32_t>(lead_headers->size()), h2::kHeaders, h2::kFlagEndHeaders, stream);
    iov.push_back({lh, 9});
    if (!lead_headers->empty()) iov.push_back({const_cast<char*>(lead_headers->data()), lead_headers->size()});
  }
  iov.push_back({hdr, 9});
  WriteLock lk(*this);
  if (type == h2::kData) note_data_frame();
  for (size_t i = 0; i < pieces.size(); ++i) {
    const SendPiece& p = pieces[i];
    if (p.fd < 0 && !p.splice) {
      if (p.n) iov.push_back({const_cast<uint8_t*>(p.p), p.n});
      continue;
    }
    if (!iov.empty()) {
      conn_.writev_all(iov.data(), static_cast<int>(iov.size()), /*more=*/true);
      iov.clear();
    }
    if (p.splice)
      conn_.splice_user_all(p.p, p.n, /*more=*/i + 1 < pieces.size() || trailers);
    else
      conn_.sendfile_all(p.fd, p.foff, p.n, /*more=*/false);
  }
  if (trailers) {
    encode_frame_header(th, static_cast<uint32_t>(trailers->size()), h2::kHeaders,
                        h2::kFlagEndHeaders | h2::kFlagEndStream, stream);
    iov.push_back({th, 9});
    if (!trailers->empty()) iov.push_back({const_cast<char*>(trailers->data()), trailers->size()});
  }
  if (!iov.empty()) conn_.writev_all(iov.data(), static_cast<int>(iov.size()));
}

void H2Writer::write_data_train(uint32_t stream, const std::vector<SendPiece>& pieces, size_t total,
                                uint8_t last_flags, const std::string* lead_headers, const std::string* trailers) {
  const size_t fmax = std::max<size_t>(1, peer_max_frame_.load());
  bool any_fd = false;
  for (const SendPiece& p : pieces) any_fd |= p.fd >= 0 && p.n > 0;
  if (any_fd || total <= fmax || fmax >= kTrainCopyMaxFrame) {
    // one frame, large frames or sendfile pieces: frame by frame (zero copy)
    size_t idx = 0, off = 0, left = total;
    bool first = true;
    std::vector<SendPiece> frame;
    do {
      const size_t n = std::min(left, fmax);
      frame.clear();
      for (size_t need = n; need > 0;) {
        const SendPiece& src = pieces[idx];
        SendPiece q = src;
        const size_t k = std::min(need, src.n - off);
        q.p = src.p ? src.p + off : nullptr;
        q.foff = src.foff + off;
        q.n = k;
        if (k) frame.push_back(q);
        need -= k;
        off += k;
        if (off == src.n) {
          ++idx;
          off = 0;
        }
      }
      left -= n;
      write_frame_pieces(h2::kData, left == 0 ? last_flags : 0, stream, frame, n, first ? lead_headers : nullptr,
                         left == 0 ? trailers : nullptr);
      first = false;
    } while (left > 0);
    return;
  }
  const size_t nframes = (total + fmax - 1) / fmax;
  std::vector<iovec> iov;
  iov.reserve(pieces.size() + 3 * nframes + 4);
  std::vector<uint8_t> hdrs(9 * (nframes + 2));  // the headers live here until the write
  size_t hpos = 0;
  auto header = [&](uint32_t len, uint8_t type, uint8_t flags) {
    uint8_t* h = &hdrs[hpos];
    hpos += 9;
    encode_frame_header(h, len, type, flags, stream);
    iov.push_back({h, 9});
  };
  if (lead_headers) {
    header(static_cast<uint32_t>(lead_headers->size()), h2::kHeaders, h2::kFlagEndHeaders);
    if (!lead_headers->empty()) iov.push_back({const_cast<char*>(lead_headers->data()), lead_headers->size()});
  }
  size_t idx = 0, off = 0, left = total, frames = 0;
  while (left > 0) {
    const size_t n = std::min(left, fmax);
    left -= n;
    header(static_cast<uint32_t>(n), h2::kData, left == 0 ? last_flags : 0);
    ++frames;
    for (size_t need = n; need > 0;) {
      const SendPiece& src = pieces[idx];
      const size_t k = std::min(need, src.n - off);
      if (k) iov.push_back({const_cast<uint8_t*>(src.p + off), k});
      need -= k;
      off += k;
      if (off == src.n) {
        ++idx;
        off = 0;
      }
    }
  }
  if (trailers) {
    header(static_cast<uint32_t>(trailers->size()), h2::kHeaders, h2::kFlagEndHeaders | h2::kFlagEndStream);
    if (!trailers->empty()) iov.push_back({const_cast<char*>(trailers->data()), trailers->size()});
  }
  WriteLock lk(*this);
  for (size_t i = 0; i < frames; ++i) note_data_frame();
  conn_.writev_all(iov.data(), static_cast<int>(iov.size()));
}

void H2Writer::write_headers(uint32_t stream, const std::string& block, bool end_stream) {
  const size_t maxf = peer_max_frame_;
  WriteLock lk(*this);  // HEADERS+CONTINUATION must be contiguous
  size_t off = 0;
  bool first = true;
  do {
    size_t n = std::min(maxf, block.size() - off);
    bool last = off + n == block.size();
    uint8_t flags = (last ? h2::kFlagEndHeaders : 0) | (first && end_stream ? h2::kFlagEndStream : 0);
    uint8_t hdr[9];
    encode_frame_header(hdr, static_cast<uint32_t>(n), first ? h2::kHeaders : h2::kContinuation, flags, stream);
    iovec iov[2] = {{hdr, 9}, {const_cast<char*>(block.data() + off), n}};
    conn_.writev_all(iov, n ? 2 : 1);
    off += n;
    first = false;
  } while (off < block.size());
}

bool H2Writer::write_headers_and_data(uint32_t stream, const std::string& block, const uint8_t* p, size_t n) {
  {
    std::lock_guard<std::mutex> lk(fmu_);
    auto it = stream_window_.find(stream);
    if (dead_ || it == stream_window_.end() || block.size() > peer_max_frame_ || n > peer_max_frame_ ||
        static_cast<int64_t>(n) > std::min(conn_window_, it->second))
      return false;
    conn_window_ -= static_cast<int64_t>(n);
    it->second -= static_cast<int64_t>(n);
  }
  uint8_t hh[9], dh[9];
  encode_frame_header(hh, static_cast<uint32_t>(block.size()), h2::kHeaders, h2::kFlagEndHeaders, stream);
  encode_frame_header(dh, static_cast<uint32_t>(n), h2::kData, h2::kFlagEndStream, stream);
  iovec iov[4] = {{hh, 9}, {const_cast<char*>(block.data()), block.size()}, {dh, 9}, {const_cast<uint8_t*>(p), n}};
  WriteLock lk(*this);
  conn_.writev_all(iov, 4);
  return true;
}

void H2Writer::write_window_update(uint32_t stream, uint32_t inc) {
  uint8_t v[4];
  put_be32(v, inc & 0x7FFFFFFF);
  write_control(h2::kWindowUpdate, 0, stream, v, 4);
}

void H2Writer::write_rst(uint32_t stream, uint32_t code) {
  uint8_t v[4];
  put_be32(v, code);
  write_frame(h2::kRstStream, 0, stream, v, 4);
}

void H2Writer::write_goaway(uint32_t last_stream, uint32_t code, const std::string& msg) {
  std::string p(8, '\0');
  put_be32(reinterpret_cast<uint8_t*>(&p[0]), last_stream & 0x7FFFFFFF);
  put_be32(reinterpret_cast<uint8_t*>(&p[4]), code);
  p += msg;
  write_frame(h2::kGoaway, 0, 0, p.data(), p.size());
}

size_t H2Writer::reserve(uint32_t stream, size_t want) {
  std::unique_lock<std::mutex> lk(fmu_);
  for (;;) {
    if (dead_) return 0;
    auto it = stream_window_.find(stream);
    if (it == stream_window_.end()) return 0;
    int64_t avail = std::min(conn_window_, it->second);
    if (avail > 0) {
      size_t n = std::min<size_t>({want, static_cast<size_t>(avail), static_cast<size_t>(peer_max_frame_.load())});
      if (quantum_ > 0 && stream_window_.size() > 1) n = std::min(n, quantum_);
      conn_window_ -= static_cast<int64_t>(n);
      it->second -= static_cast<int64_t>(n);
      return n;
    }
    fcv_.wait(lk);
  }
}

size_t H2Writer::try_reserve(uint32_t stream, size_t want, bool* gone) {
  std::lock_guard<std::mutex> lk(fmu_);
  *gone = false;
  auto it = stream_window_.find(stream);
  if (dead_ || it == stream_window_.end()) {
    *gone = true;
    return 0;
  }
  const int64_t avail = std::min(conn_window_, it->second);
  if (avail <= 0) return 0;
  const size_t n = std::min<size_t>({want, static_cast<size_t>(avail), static_cast<size_t>(peer_max_frame_.load())});
  conn_window_ -= static_cast<int64_t>(n);
  it->second -= static_cast<int64_t>(n);
  return n;
}

size_t H2Writer::train_grant_locked(int64_t avail, size_t want) const {
  size_t n = std::min<size_t>(want, static_cast<size_t>(avail));
  const size_t fmax = peer_max_frame_.load();
  if (n < want && n > fmax) n -= n % fmax;
  return n;
}

size_t H2Writer::reserve_train(uint32_t stream, size_t want) {
  std::unique_lock<std::mutex> lk(fmu_);
  for (;;) {
    if (dead_) return 0;
    auto it = stream_window_.find(stream);
    if (it == stream_window_.end()) return 0;
    const int64_t avail = std::min(conn_window_, it->second);
    if (avail > 0) {
      size_t w = want;
      if (quantum_ > 0 && stream_window_.size() > 1) w = std::min(w, quantum_);
      const size_t n = train_grant_locked(avail, w);
      conn_window_ -= static_cast<int64_t>(n);
      it->second -= static_cast<int64_t>(n);
      return n;
    }
    fcv_.wait(lk);
  }
}

size_t H2Writer::try_reserve_train(uint32_t stream, size_t want, bool* gone) {
  std::lock_guard<std::mutex> lk(fmu_);
  *gone = false;
  auto it = stream_window_.find(stream);
  if (dead_ || it == stream_window_.end()) {
    *gone = true;
    return 0;
  }
  const int64_t avail = std::min(conn_window_, it->second);
  if (avail <= 0) return 0;
  const size_t n = train_grant_locked(avail, want);
  conn_window_ -= static_cast<int64_t>(n);
  it->second -= static_cast<int64_t>(n);
  return n;
}

void H2Writer::wait_window(int timeout_ms) {
  std::unique_lock<std::mutex> lk(fmu_);
  fcv_.wait_for(lk, std::chrono::milliseconds(timeout_ms));
}

void H2Writer::register_stream(uint32_t stream) {
  std::lock_guard<std::mutex> lk(fmu_);
  stream_window_[stream] = peer_initial_window_.load();
}

void H2Writer::unregister_stream(uint32_t stream) {
  std::lock_guard<std::mutex> lk(fmu_);
  stream_window_.erase(stream);
  fcv_.notify_all();
}

void H2Writer::on_window_update(uint32_t stream, uint32_t inc) {
  std::lock_guard<std::mutex> lk(fmu_);
  if (stream == 0) {
    conn_window_ += inc;
  } else {
    auto it = stream_window_.find(stream);
    if (it != stream_window_.end()) it->second += inc;
  }
  fcv_.notify_all();
}

void H2Writer::on_peer_settings(const H2Settings& s, uint32_t old_initial_window) {
  std::lock_guard<std::mutex> lk(fmu_);
  int64_t delta = static_cast<int64_t>(s.initial_window_size) - static_cast<int64_t>(old_initial_window);
  if (delta)
    for (auto& kv : stream_window_) kv.second += delta;
  peer_initial_window_ = s.initial_window_size;
  peer_max_frame_ = s.max_frame_size;
  fcv_.notify_all();
}

void H2Writer::kill() {
  std::lock_guard<std::mutex> lk(fmu_);
  dead_ = true;
  fcv_.notify_all();
}

}  // namespace gcsb
