#include "net/buffered.h"

#include <stdexcept>

#include "core/util.h"

namespace gcsb {

std::string BufferedConn::read_line(size_t max) {
  if (arena_) throw std::logic_error("BufferedConn::read_line in arena mode (HTTP/1.1 never uses an arena)");
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

}  // namespace gcsb
