// Buffered reader over a Conn: small reads (HTTP header lines, HTTP/2 frame
// headers, protobuf tags) are served from a 16 KiB buffer, large payload reads
// bypass it and recv() straight into the caller's memory (the pinned ring slot
// when the GPU sink is active), so object bytes are copied exactly once by the
// kernel from socket buffers to their landing memory.
#pragma once
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <utility>

#include <sys/types.h>

#include "core/util.h"
#include "net/socket.h"

namespace gcsb {

// Receive memory owned by someone else (the GPU sink's connection ring,
// gpu/engine.h ConnRing): a BufferedConn in arena mode recv()s straight into
// it, as much as the window holds, and parses protocol bytes in place;
// payload is handed to the sink where it already lies (take_inplace), so one
// recv() crosses frame and message boundaries and no byte goes through a
// bounce buffer.  Only the connection's reader thread calls these.
class RecvArena {
 public:
  virtual ~RecvArena() = default;
  // Writable memory for the next recv() (blocks until the arena has room).
  // Called only when every byte of the previous windows was consumed.
  virtual std::pair<uint8_t*, size_t> recv_window() = 0;
  // n bytes were received at the start of the last window.
  virtual void received(size_t n) = 0;
};

class BufferedConn {
 public:
  explicit BufferedConn(std::unique_ptr<Conn> c, RecvArena* arena = nullptr)
      : conn_(std::move(c)), buf_(arena ? nullptr : new uint8_t[kCap]), arena_(arena) {}
  Conn& conn() { return *conn_; }
  bool is_open() const { return conn_ && conn_->is_open(); }
  size_t buffered() const { return end_ - pos_; }
  // arena mode: payload can be taken in place (take_inplace)
  bool inplace() const { return arena_ != nullptr; }

  // Up to n payload bytes where they lie in the arena (arena mode only): a
  // recv() happens only when nothing is buffered, and it fills the whole
  // window.  Returns the count (>= 1) and sets *p.
  size_t take_inplace(size_t n, const uint8_t** p) {
    if (!buffered()) afill();
    const size_t b = buffered() < n ? buffered() : n;
    *p = abuf_ + pos_;
    pos_ += b;
    return b;
  }

  // Read exactly n bytes (n small or large).
  void read_exact(void* dst, size_t n) {
    if (arena_) {
      auto* d = static_cast<uint8_t*>(dst);
      while (n) {
        if (!buffered()) afill();
        const size_t b = buffered() < n ? buffered() : n;
        std::memcpy(d, abuf_ + pos_, b);
        pos_ += b;
        d += b;
        n -= b;
      }
      return;
    }
    auto* d = static_cast<uint8_t*>(dst);
    size_t b = buffered() < n ? buffered() : n;
    if (b) {
      std::memcpy(d, buf_.get() + pos_, b);
      pos_ += b;
      d += b;
      n -= b;
    }
    if (n == 0) return;
    if (n < 512) {  // small: refill the buffer
      while (buffered() < n) fill();
      std::memcpy(d, buf_.get() + pos_, n);
      pos_ += n;
    } else {
      conn_->read_exact(d, n);
    }
  }
  // Read 1..n bytes directly (large-payload path). Returns 0 only on EOF.
  // SocketOptions::recv_refill: a large read also refills this buffer in the
  // same recvmsg(), so whatever follows the payload (the next frame header)
  // is parsed without a system call of its own.  Round 3 saw half the
  // receive calls and no rate change under the pacing-timer noise
  // (profiles/r3_refill); HTTP bodies pay a 16 KiB bounce per read.
  size_t read_some(void* dst, size_t n) {
    if (arena_) {  // a sink that cannot take bytes in place: copy them out
      if (!buffered()) afill();
      const size_t b = buffered() < n ? buffered() : n;
      std::memcpy(dst, abuf_ + pos_, b);
      pos_ += b;
      return b;
    }
    if (buffered()) {
      size_t b = buffered() < n ? buffered() : n;
      std::memcpy(dst, buf_.get() + pos_, b);
      pos_ += b;
      return b;
    }
    if (n >= kRefillMin && conn_->recv_refill()) {
      pos_ = end_ = 0;
      const size_t r = conn_->read_some2(dst, n, buf_.get(), fill_cap());
      if (r <= n) return r;
      end_ = r - n;
      return n;
    }
    return conn_->read_some(dst, n);
  }
  // Scatter receive for the HTTP/2 reader's frame spanning
  // (h2/h2_client.h H2DataCursor::read_spanning): ONE recvmsg() into
  // iov[0..cnt) and then this buffer (whatever follows the plan, e.g. the
  // next frame's header).  Needs an empty buffer; returns the bytes that
  // landed in iov (any past them are buffered now).  TLS: iov[0] alone.
  size_t recv_scatter(struct iovec* iov, int cnt);
  // Puts n bytes back in front of the buffered ones: a scatter plan that
  // guessed a frame boundary wrong hands the bytes after it back to the
  // parser (the buffer grows if they do not fit).
  void unread(const uint8_t* p, size_t n);
  void skip(size_t n) {
    uint8_t tmp[4096];
    while (n) {
      size_t k = n < sizeof(tmp) ? n : sizeof(tmp);
      read_exact(tmp, k);
      n -= k;
    }
  }
  uint8_t read_byte() {
    if (arena_) {
      if (!buffered()) afill();
      return abuf_[pos_++];
    }
    if (!buffered()) fill();
    return buf_[pos_++];
  }
  // Reads a CRLF/LF-terminated line (without terminator). Throws if > max.
  std::string read_line(size_t max = 65536);

 private:
  static constexpr size_t kCap = 16384;
  static constexpr size_t kRefillMin = 64u << 10;
  void fill() {
    if (pos_ == end_) pos_ = end_ = 0;
    if (end_ == cap_) {
      std::memmove(buf_.get(), buf_.get() + pos_, end_ - pos_);
      end_ -= pos_;
      pos_ = 0;
    }
    const size_t room = cap_ - end_;
    size_t r = conn_->read_some(buf_.get() + end_, room < fill_cap() ? room : fill_cap());
    if (r == 0) throw StorageError("unexpected EOF", true);
    end_ += r;
  }
  size_t fill_cap() const {
    const size_t f = conn_->fill_bytes();
    return f < 64 ? 64 : (f > kCap ? kCap : f);
  }
  // arena mode: the next window, filled by one recv()
  void afill() {
    auto w = arena_->recv_window();
    const size_t r = conn_->read_some(w.first, w.second);
    if (r == 0) throw StorageError("unexpected EOF", true);
    arena_->received(r);
    abuf_ = w.first;
    pos_ = 0;
    end_ = r;
  }
  std::unique_ptr<Conn> conn_;
  std::unique_ptr<uint8_t[]> buf_;
  RecvArena* arena_ = nullptr;
  uint8_t* abuf_ = nullptr;  // arena mode: start of the current window
  size_t cap_ = kCap;        // buf_'s size (unread() may grow it)
  size_t pos_ = 0, end_ = 0;
};

}  // namespace gcsb
