#include "core/content.h"

#include <cstdlib>

#include <sys/mman.h>

#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <stdexcept>
#include <thread>

#include "core/affinity.h"
#include "core/crc32c.h"
#include "core/hugebuf.h"

namespace gcsb {

namespace {
constexpr uint64_t kBlock = 64 << 10;

struct ShiftBlock {
  uint32_t tab[4][256];
  ShiftBlock() { crc32c_build_shift_table(kBlock, tab); }
};
const ShiftBlock& shift_block() {
  static ShiftBlock s;
  return s;
}
}  // namespace

uint64_t object_rotation(const std::string& name) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (unsigned char c : name) {
    h ^= c;
    h *= 0x100000001B3ull;
  }
  return h % (kPatternLen / kPatternRotAlign) * kPatternRotAlign;
}

PatternBuffer::PatternBuffer() {
  const uint64_t total = kPatternLen + kPatternExt;
  buf_.resize(total);
  // generate kPatternLen bytes in parallel, then copy the wrap extension
  const unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  const uint64_t words = kPatternLen / 8;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) {
    th.emplace_back([&, t] {
      uint64_t w0 = words * t / nt, w1 = words * (t + 1) / nt;
      for (uint64_t w = w0; w < w1; ++w) {
        uint64_t v = splitmix64_at(kPatternSeed, w);
        std::memcpy(&buf_[w * 8], &v, 8);
      }
    });
  }
  for (auto& x : th) x.join();
  for (uint64_t i = words * 8; i < kPatternLen; ++i) buf_[i] = pattern_byte(kPatternSeed, i);
  std::memcpy(&buf_[kPatternLen], &buf_[0], kPatternExt);
  const uint64_t nblocks = kPatternLen / kBlock;
  block_crc_.resize(nblocks);
  for (uint64_t b = 0; b < nblocks; ++b) block_crc_[b] = crc32c(&buf_[b * kBlock], kBlock);
}

int PatternBuffer::memfd() const {
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  if (memfd_ != -2) return memfd_;
  int fd = static_cast<int>(::syscall(SYS_memfd_create, "gcsb-pattern", 0));
  if (fd >= 0) {
    size_t off = 0;
    while (off < buf_.size()) {
      ssize_t w = ::write(fd, buf_.data() + off, buf_.size() - off);
      if (w <= 0) {
        ::close(fd);
        fd = -1;
        break;
      }
      off += static_cast<size_t>(w);
    }
  }
  memfd_ = fd;
  return memfd_;
}

const uint8_t* PatternBuffer::thp() const {
  // every body send asks: after the first call a plain atomic load, no lock
  std::call_once(thp_once_, [this] {
    try {
      uint8_t* p = huge_alloc(buf_.size());  // faulted in here: on this thread's node
      std::memcpy(p, buf_.data(), buf_.size());
      thp_.store(p, std::memory_order_release);
    } catch (const std::bad_alloc&) {
    }
  });
  return thp_.load(std::memory_order_acquire);
}

std::vector<long> PatternBuffer::memfd_numa() const {
  if (const uint8_t* t = thp_.load(std::memory_order_acquire)) return numa_nodes_of(t, buf_.size());
  if (memfd_ < 0) return {};
  void* m = ::mmap(nullptr, buf_.size(), PROT_READ, MAP_SHARED | MAP_POPULATE, memfd_, 0);
  if (m == MAP_FAILED) return {};
  std::vector<long> c = numa_nodes_of(m, buf_.size());
  ::munmap(m, buf_.size());
  return c;
}

const PatternBuffer& PatternBuffer::instance() {
  static PatternBuffer* pb = new PatternBuffer();
  return *pb;
}

const uint8_t* PatternBuffer::slice(uint64_t rot, uint64_t off, uint64_t n) const {
  if (n > kPatternExt) throw std::runtime_error("pattern slice too long");
  return buf_.data() + (off + rot) % kPatternLen;
}

uint32_t PatternBuffer::crc32c_range(uint64_t rot, uint64_t off, uint64_t n) const {
  uint32_t crc = 0;
  uint64_t p = (off + rot) % kPatternLen;
  const ShiftBlock& sb = shift_block();
  while (n > 0) {
    uint64_t piece = std::min<uint64_t>(n, kPatternLen - p);
    // [p, p+piece) lies inside the pattern proper
    uint64_t a = p, e = p + piece;
    uint64_t first_full = (a + kBlock - 1) / kBlock * kBlock;
    if (first_full > e) first_full = e;
    crc = crc32c_extend(crc, &buf_[a], first_full - a);
    a = first_full;
    uint64_t nblocks = kPatternLen / kBlock;
    while (a + kBlock <= e && a / kBlock < nblocks) {
      crc = crc32c_apply_shift_table(sb.tab, crc) ^ block_crc_[a / kBlock];
      a += kBlock;
    }
    crc = crc32c_extend(crc, &buf_[a], e - a);
    n -= piece;
    p = 0;
  }
  return crc;
}

void fill_object_bytes(uint8_t* dst, uint64_t rot, uint64_t off, uint64_t n) {
  const PatternBuffer& pb = PatternBuffer::instance();
  while (n > 0) {
    uint64_t piece = std::min<uint64_t>(n, kPatternExt);
    std::memcpy(dst, pb.slice(rot, off, piece), piece);
    dst += piece;
    off += piece;
    n -= piece;
  }
}

}  // namespace gcsb
