#include "storage/pipe_relay.h"

#include <fcntl.h>
#include <poll.h>
#include <sys/ioctl.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <stdexcept>

#include "core/hugebuf.h"
#include "core/util.h"

namespace gcsb {

namespace {

std::atomic<uint64_t> g_relays{0}, g_no_pipe{0}, g_spliced{0}, g_splices{0}, g_buffered{0}, g_overflow{0},
    g_overflows{0}, g_pipes{0}, g_pipe_bytes{0};

constexpr size_t kBlock = 2u << 20;  // overflow block (one THP)
constexpr int kMaxBlocks = 4;        // beyond this the reader waits for the pipe instead

// LIFO pool: the pipe handed back most recently goes out first.
std::mutex g_pool_mu;
std::vector<RelayPipe> g_pool;
int g_live = 0;  // pipes in existence (pooled + in use)

void close_pipe(RelayPipe& p) {
  if (p.r >= 0) ::close(p.r);
  if (p.w >= 0) ::close(p.w);
  p = RelayPipe{};
}

RelayPipe take_pipe() {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_pool.empty()) {
      RelayPipe p = g_pool.back();
      g_pool.pop_back();
      return p;
    }
    if (g_live >= PipeRelay::kMaxPipes) return RelayPipe{};
    ++g_live;
  }
  RelayPipe p;
  int fds[2];
  if (::pipe2(fds, O_CLOEXEC) == 0) {
    p.r = fds[0];
    p.w = fds[1];
    // the write end never blocks the connection's reader: a full pipe
    // overflows into a block instead (PipeRelay::feed)
    (void)::fcntl(p.w, F_SETFL, O_NONBLOCK);
    // 1 MiB is fs.pipe-max-size's default, the most an unprivileged process
    // may ask; the user's pipe-page budget may allow less
    for (int sz = 1 << 20; sz >= static_cast<int>(PipeRelay::kMinPipe); sz >>= 1)
      if (::fcntl(p.w, F_SETPIPE_SZ, sz) >= 0) break;
    const int c = ::fcntl(p.w, F_GETPIPE_SZ);
    p.cap = c > 0 ? static_cast<size_t>(c) : 0;
    if (p.cap < PipeRelay::kMinPipe) close_pipe(p);
  }
  if (p.r < 0) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    --g_live;
    return p;
  }
  g_pipes.fetch_add(1, std::memory_order_relaxed);
  g_pipe_bytes.fetch_add(p.cap, std::memory_order_relaxed);
  return p;
}

void give_pipe(RelayPipe p, bool clean) {
  int queued = 0;
  if (clean && (::ioctl(p.r, FIONREAD, &queued) != 0 || queued != 0)) clean = false;
  if (!clean) {
    close_pipe(p);  // stray bytes: never hand them to the next read
    std::lock_guard<std::mutex> lk(g_pool_mu);
    --g_live;
    return;
  }
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool.push_back(p);
}

}  // namespace

PipeRelayStats pipe_relay_stats() {
  PipeRelayStats s;
  s.relays = g_relays.load();
  s.no_pipe = g_no_pipe.load();
  s.spliced_bytes = g_spliced.load();
  s.splices = g_splices.load();
  s.buffered_bytes = g_buffered.load();
  s.overflow_bytes = g_overflow.load();
  s.overflows = g_overflows.load();
  s.pipes = g_pipes.load();
  s.pipe_bytes = g_pipe_bytes.load();
  return s;
}

PipeRelay::PipeRelay(Sink& inner) : inner_(inner), pipe_(take_pipe()) {
  (usable() ? g_relays : g_no_pipe).fetch_add(1, std::memory_order_relaxed);
}

PipeRelay::~PipeRelay() {
  // settle() is the normal end; here only what an exception path left
  std::lock_guard<std::mutex> c(cmu_);
  std::lock_guard<std::mutex> q(qmu_);
  for (const Op& op : ops_)
    if (op.kind == Op::kRelease) huge_give(op.p, kBlock);
  ops_.clear();
  if (blk_) huge_give(blk_, kBlock);
  blk_ = nullptr;
  if (pipe_.r >= 0) give_pipe(pipe_, false);
}

void PipeRelay::push(Op op) {
  std::lock_guard<std::mutex> q(qmu_);
  ops_.push_back(std::move(op));
}

size_t PipeRelay::feed(BufferedConn& bc, size_t n) {
  if (pipe_dirty_.load(std::memory_order_acquire)) {  // the read has failed: drop its payload
    bc.skip(n);
    return n;
  }
  for (;;) {
    const bool from_buffer = bc.buffered() > 0;
    const ssize_t m = bc.splice_some(pipe_.w, n);
    if (m > 0) {
      if (from_buffer) {
        g_buffered.fetch_add(static_cast<uint64_t>(m), std::memory_order_relaxed);
      } else {
        g_spliced.fetch_add(static_cast<uint64_t>(m), std::memory_order_relaxed);
        g_splices.fetch_add(1, std::memory_order_relaxed);
      }
      Op op{Op::kPipe};
      op.len = static_cast<size_t>(m);
      push(std::move(op));
      return static_cast<size_t>(m);
    }
    if (m == 0) return 0;
    // the pipe is full: this stream's worker is behind
    if (blocks_.load(std::memory_order_acquire) >= kMaxBlocks && !blk_) {
      // far behind: wait for room rather than buffer without bound
      pollfd pfd{pipe_.w, POLLOUT, 0};
      (void)::poll(&pfd, 1, 100);
      if (pipe_dirty_.load(std::memory_order_acquire)) {
        bc.skip(n);
        return n;
      }
      continue;
    }
    if (!blk_) {
      blk_ = huge_take(kBlock);
      blk_used_ = 0;
      blocks_.fetch_add(1, std::memory_order_relaxed);
    }
    const size_t k = bc.read_some(blk_ + blk_used_, std::min(n, kBlock - blk_used_));
    if (k == 0) return 0;
    Op op{Op::kCopy};
    op.p = blk_ + blk_used_;
    op.len = k;
    blk_used_ += k;
    push(std::move(op));
    if (blk_used_ == kBlock) {
      Op rel{Op::kRelease};
      rel.p = blk_;
      push(std::move(rel));
      blk_ = nullptr;
    }
    g_overflow.fetch_add(k, std::memory_order_relaxed);
    g_overflows.fetch_add(1, std::memory_order_relaxed);
    return k;
  }
}

void PipeRelay::begin(const ObjectInfo& info) {
  Op op{Op::kOpen};
  op.info = info;
  push(std::move(op));
}

void PipeRelay::update_info(const ObjectInfo& info) {
  Op op{Op::kInfo};
  op.info = info;
  push(std::move(op));
}

void PipeRelay::chunk_begin(size_t len) {
  Op op{Op::kBegin};
  op.len = len;
  push(std::move(op));
}

void PipeRelay::chunk_end(bool has_crc, uint32_t crc) {
  Op op{Op::kEnd};
  op.has_crc = has_crc;
  op.crc = crc;
  push(std::move(op));
}

Window PipeRelay::acquire(size_t) { throw std::logic_error("PipeRelay: payload goes through feed()"); }
void PipeRelay::commit(size_t) { throw std::logic_error("PipeRelay: payload goes through feed()"); }

void PipeRelay::fail(const char* what) {
  if (failed_) return;
  failed_ = true;
  if (on_error_) on_error_(std::string("sink: ") + what);
}

size_t PipeRelay::read_pipe(uint8_t* dst, size_t n) {
  for (;;) {
    const ssize_t r = ::read(pipe_.r, dst, n);
    if (r > 0) return static_cast<size_t>(r);
    if (r < 0 && errno == EINTR) continue;
    // every byte counted in an op is in the pipe: this cannot happen short of
    // a broken pipe.  Fail the read, stop reading the pipe (the reader then
    // drops this stream's payload) and leave the pipe out of the pool.
    pipe_dirty_.store(true, std::memory_order_release);
    fail(r < 0 ? "relay pipe read failed" : "relay pipe read: EOF");
    return 0;
  }
}

void PipeRelay::pipe_into_sink(size_t n) {
  while (n > 0) {
    if (pipe_dirty_.load(std::memory_order_relaxed)) return;
    if (failed_) {
      if (scratch_.size() < (64u << 10)) scratch_.resize(64u << 10);
      n -= read_pipe(scratch_.data(), std::min(n, scratch_.size()));
      continue;
    }
    Window w;
    try {
      w = inner_.acquire(n);
    } catch (const std::exception& e) {
      fail(e.what());
      continue;
    }
    const size_t k = read_pipe(w.ptr, std::min(n, w.cap));
    if (k == 0) return;
    n -= k;
    try {
      inner_.commit(k);
    } catch (const std::exception& e) {
      fail(e.what());
    }
  }
}

void PipeRelay::deliver(const uint8_t* src, size_t n) {
  while (n > 0 && !failed_) {
    try {
      Window w = inner_.acquire(n);
      const size_t k = std::min(n, w.cap);
      std::memcpy(w.ptr, src, k);
      inner_.commit(k);
      src += k;
      n -= k;
    } catch (const std::exception& e) {
      fail(e.what());
    }
  }
}

void PipeRelay::apply(const Op& op) {
  switch (op.kind) {
    case Op::kPipe:
      pipe_into_sink(op.len);
      return;
    case Op::kCopy:
      deliver(op.p, op.len);
      return;
    case Op::kRelease:
      huge_give(op.p, kBlock);
      blocks_.fetch_sub(1, std::memory_order_release);
      return;
    default:
      break;
  }
  if (failed_) return;
  try {
    if (op.kind == Op::kOpen) inner_.begin(op.info);
    else if (op.kind == Op::kInfo) inner_.update_info(op.info);
    else if (op.kind == Op::kBegin) inner_.chunk_begin(op.len);
    else inner_.chunk_end(op.has_crc, op.crc);
  } catch (const std::exception& e) {
    fail(e.what());
  }
}

void PipeRelay::drain() {
  std::lock_guard<std::mutex> c(cmu_);
  for (;;) {
    batch_.clear();
    {
      std::lock_guard<std::mutex> q(qmu_);
      if (ops_.empty()) break;
      batch_.swap(ops_);
    }
    for (const Op& op : batch_) apply(op);
  }
  if (inner_.deferred() && !failed_) inner_.drain();
}

void PipeRelay::settle() {
  if (blk_) {  // the reader is done with this relay: its last block goes back after its bytes
    Op rel{Op::kRelease};
    rel.p = blk_;
    push(std::move(rel));
    blk_ = nullptr;
  }
  drain();
  std::lock_guard<std::mutex> c(cmu_);
  if (pipe_.r >= 0) give_pipe(pipe_, !pipe_dirty_.load());
  pipe_ = RelayPipe{};
}

SinkResult PipeRelay::finish() {
  settle();
  return inner_.finish();
}

void PipeRelay::abort() {
  settle();
  inner_.abort();
}

}  // namespace gcsb
