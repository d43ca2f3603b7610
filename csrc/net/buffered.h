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
  // SocketOptions::recv_refill: a large read also refills this buffer in the
  // same recvmsg(), so whatever follows the payload (the next frame header)
  // is parsed without a system call of its own.  Round 3 saw half the
  // receive calls and no rate change under the pacing-timer noise
  // (profiles/r3_refill); HTTP bodies pay a 16 KiB bounce per read.
  size_t read_some(void* dst, size_t n) {
    if (buffered()) {
      size_t b = buffered() < n ? buffered() : n;
      std::memcpy(dst, buf_.get() + pos_, b);
      pos_ += b;
      return b;
    }
    if (n >= kRefillMin && conn_->recv_refill()) {
      pos_ = end_ = 0;
      const size_t r = conn_->read_some2(dst, n, buf_.get(), kCap);
      if (r <= n) return r;
      end_ = r - n;
      return n;
    }
    return conn_->read_some(dst, n);
  }
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
  static constexpr size_t kRefillMin = 64u << 10;
  void fill() {
    if (pos_ == end_) pos_ = end_ = 0;
    if (end_ == kCap) {
      std::memmove(buf_.get(), buf_.get() + pos_, end_ - pos_);
      end_ -= pos_;
      pos_ = 0;
    }
    size_t r = conn_->read_some(buf_.get() + end_, kCap - end_);
    if (r == 0) throw StorageError("unexpected EOF", true);
    end_ += r;
  }
  std::unique_ptr<Conn> conn_;
  std::unique_ptr<uint8_t[]> buf_;
  size_t pos_ = 0, end_ = 0;
};

}  // namespace gcsb
