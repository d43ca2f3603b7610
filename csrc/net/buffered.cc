#include "net/buffered.h"

#include <sys/uio.h>

#include <stdexcept>
#include <vector>

#include "core/util.h"

namespace gcsb {

std::string BufferedConn::read_line(size_t max) {
  std::string line;
  for (;;) {
    if (!buffered()) fill();
    const uint8_t* s = buf_.get() + pos_;
    size_t avail = buffered();
    const void* nl = std::memchr(s, '\n', avail);
    if (nl) {
      size_t k = static_cast<const uint8_t*>(nl) - s;
      line.append(reinterpret_cast<const char*>(s), k);
      pos_ += k + 1;
      if (!line.empty() && line.back() == '\r') line.pop_back();
      return line;
    }
    line.append(reinterpret_cast<const char*>(s), avail);
    pos_ += avail;
    if (line.size() > max) throw StorageError("header line too long", false);
  }
}

size_t BufferedConn::recv_scatter(struct iovec* iov, int cnt) {
  if (buffered()) throw std::logic_error("BufferedConn::recv_scatter needs an empty buffer");
  pos_ = end_ = 0;
  if (conn_->tls()) {
    const size_t r = conn_->read_some(iov[0].iov_base, iov[0].iov_len);
    if (r == 0) throw StorageError("unexpected EOF", true);
    return r;
  }
  std::vector<iovec> v(iov, iov + cnt);
  size_t plan = 0;
  for (int i = 0; i < cnt; ++i) plan += iov[i].iov_len;
  v.push_back({buf_.get(), fill_cap()});
  const size_t r = conn_->read_somev(v.data(), static_cast<int>(v.size()));
  if (r == 0) throw StorageError("unexpected EOF", true);
  if (r > plan) {
    end_ = r - plan;
    return plan;
  }
  return r;
}

void BufferedConn::unread(const uint8_t* p, size_t n) {
  if (n == 0) return;
  const size_t have = buffered();
  if (n + have > cap_) {
    size_t cap = cap_ * 2;
    while (cap < n + have) cap *= 2;
    std::unique_ptr<uint8_t[]> nb(new uint8_t[cap]);
    std::memcpy(nb.get() + n, buf_.get() + pos_, have);
    buf_ = std::move(nb);
    cap_ = cap;
  } else {
    std::memmove(buf_.get() + n, buf_.get() + pos_, have);
  }
  std::memcpy(buf_.get(), p, n);
  pos_ = 0;
  end_ = n + have;
}

}  // namespace gcsb
