// Buffered reader over a Conn: small reads (HTTP header lines, HTTP/2 frame
// headers, protobuf tags) are served from a 16 KiB buffer, large payload reads
// bypass it and recv() straight into the caller's memory (the pinned ring slot
// when the GPU sink is active), so object bytes are copied exactly once by the
// kernel from socket buffers to their landing memory.  An HTTP/2 spanning
// receive (recv_scatter) lands many frames' payload in one recvmsg().
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

class BufferedConn {
 public:
  explicit BufferedConn(std::unique_ptr<Conn> c) : conn_(std::move(c)), buf_(new uint8_t[kCap]) {}
  Conn& conn() { return *conn_; }
  bool is_open() const { return conn_ && conn_->is_open(); }
  size_t buffered() const { return end_ - pos_; }

  // Read exactly n bytes (n small or large).
  void read_exact(void* dst, size_t n) {
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
  size_t read_some(void* dst, size_t n) {
    if (buffered()) {
      size_t b = buffered() < n ? buffered() : n;
      std::memcpy(dst, buf_.get() + pos_, b);
      pos_ += b;
      return b;
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
    if (!buffered()) fill();
    return buf_[pos_++];
  }
  // Reads a CRLF/LF-terminated line (without terminator). Throws if > max.
  std::string read_line(size_t max = 65536);

 private:
  static constexpr size_t kCap = 16384;
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
  std::unique_ptr<Conn> conn_;
  std::unique_ptr<uint8_t[]> buf_;
  size_t cap_ = kCap;  // buf_'s size (unread() may grow it)
  size_t pos_ = 0, end_ = 0;
};

}  // namespace gcsb
