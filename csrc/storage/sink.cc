#include "storage/sink.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <vector>

#include "core/crc32c.h"
#include "core/hugebuf.h"
#include "core/util.h"

namespace gcsb {


DiscardSink::DiscardSink(size_t chunk_bytes, bool host_crc, bool deferred, size_t copy_out)
    : copy_out_(copy_out), cap_((chunk_bytes + 4095) / 4096 * 4096), host_crc_(host_crc),
      deferred_(deferred && host_crc) {
  if (deferred_) {
    // warm the pool with this sink's share, faulted in outside any read
    uint8_t* b[kMaxBlocks];
    for (auto& p : b) p = huge_take(cap_);
    for (auto& p : b) huge_give(p, cap_);
    return;
  }
  buf_ = huge_take(cap_);  // pooled THP (core/hugebuf.h), faulted in before any read
}

DiscardSink::~DiscardSink() {
  if (deferred_) reset_ring();
  if (buf_) huge_give(buf_, cap_);
}

void DiscardSink::reset_ring() {
  std::lock_guard<std::mutex> c(cmu_);
  std::lock_guard<std::mutex> q(qmu_);
  // every block but the current one has its kRelease op queued
  for (const Op& op : ops_)
    if (op.kind == Op::kRelease) {
      huge_give(op.blk, cap_);
      held_.fetch_sub(1, std::memory_order_relaxed);
    }
  ops_.clear();
  if (cur_) {
    huge_give(cur_, cap_);
    held_.fetch_sub(1, std::memory_order_relaxed);
    cur_ = nullptr;
  }
  cur_used_ = 0;
}

void DiscardSink::begin(const ObjectInfo& info) {
  if (deferred_) reset_ring();
  info_ = info;
  bytes_ = 0;
  obj_crc_ = 0;
  chunk_crc_ = 0;
  chunk_len_ = 0;
  in_chunk_ = false;
  chunk_partial_ = false;
  mismatch_ = false;
  any_checked_ = false;
  detail_.clear();
}

void DiscardSink::update_info(const ObjectInfo& info) {
  if (info.has_crc32c) {
    info_.has_crc32c = true;
    info_.crc32c = info.crc32c;
  }
  if (info.size >= 0) info_.size = info.size;
  if (!info.md5.empty()) info_.md5 = info.md5;
  info_.generation = info.generation;
}

Window DiscardSink::acquire(size_t want) {
  (void)want;
  if (!deferred_) return Window{buf_, cap_};
  if (cur_ && cur_used_ == cap_) {
    Op op{Op::kRelease};
    op.blk = cur_;
    push(op);
    cur_ = nullptr;
  }
  if (!cur_) {
    // backpressure: the worker fell kMaxBlocks behind, replay on this thread
    while (held_.load(std::memory_order_acquire) >= kMaxBlocks) drain();
    cur_ = huge_take(cap_);
    cur_used_ = 0;
    held_.fetch_add(1, std::memory_order_relaxed);
  }
  return Window{cur_ + cur_used_, cap_ - cur_used_};
}

void DiscardSink::push(const Op& op) {
  std::lock_guard<std::mutex> q(qmu_);
  ops_.push_back(op);
}

void DiscardSink::commit(size_t n) {
  if (deferred_) {
    Op op{Op::kData};
    op.blk = cur_;
    op.off = cur_used_;
    op.len = n;
    push(op);
    cur_used_ += n;
    bytes_ += n;
    return;
  }
  apply_data(buf_, n);
  bytes_ += n;
}

void DiscardSink::apply_data(const uint8_t* p, size_t n) {
  if (copy_out_) {
    // the consumer's Read()s: copy_out-byte copies into one small buffer
    // (io.Discard's pooled 8 KiB buffer), each read back once so the
    // copies cannot be elided
    alignas(64) static thread_local uint8_t rbuf[64 << 10];
    const size_t step = std::min(copy_out_, sizeof(rbuf));
    for (size_t o = 0; o < n; o += step) {
      const size_t k = std::min(step, n - o);
      std::memcpy(rbuf, p + o, k);
      asm volatile("" : : "r"(rbuf) : "memory");
      copy_sink_ += rbuf[k - 1];
    }
  }
  // each byte is CRC'd once: inside a chunk into the chunk CRC (combined
  // into the object CRC at chunk end), outside directly into the object CRC
  if (!host_crc_) return;
  if (in_chunk_) {
    chunk_crc_ = crc32c_extend(chunk_crc_, p, n);
    chunk_len_ += n;
  } else {
    obj_crc_ = crc32c_extend(obj_crc_, p, n);
  }
}

void DiscardSink::fold_chunk() {
  if (in_chunk_ && chunk_len_) obj_crc_ = crc32c_combine(obj_crc_, chunk_crc_, chunk_len_);
  chunk_crc_ = 0;
  chunk_len_ = 0;
}

void DiscardSink::chunk_begin(size_t) {
  if (deferred_) return push(Op{Op::kBegin});
  apply_chunk_begin();
}

void DiscardSink::apply_chunk_begin() {
  fold_chunk();
  in_chunk_ = true;
}

void DiscardSink::chunk_end(bool has_crc, uint32_t crc) {
  if (deferred_) {
    Op op{Op::kEnd};
    op.has_crc = has_crc;
    op.crc = crc;
    return push(op);
  }
  apply_chunk_end(has_crc, crc);
}

void DiscardSink::apply_chunk_end(bool has_crc, uint32_t crc) {
  if (host_crc_ && has_crc && in_chunk_ && !chunk_partial_) {
    any_checked_ = true;
    if (chunk_crc_ != crc) {
      mismatch_ = true;
      char b[128];
      std::snprintf(b, sizeof(b), "chunk crc32c mismatch: got %08x want %08x", chunk_crc_, crc);
      detail_ = b;
    }
  }
  fold_chunk();
  in_chunk_ = false;
  chunk_partial_ = false;
}

void DiscardSink::resume_at(int64_t offset) {
  (void)offset;
  if (deferred_) return push(Op{Op::kResume});
  apply_resume();
}

void DiscardSink::apply_resume() {
  // bytes of the interrupted chunk stay counted in the object CRC; the chunk
  // itself can no longer be checked on its own.
  if (in_chunk_) chunk_partial_ = true;
  fold_chunk();
  in_chunk_ = false;
}

void DiscardSink::drain() {
  if (!deferred_) return;
  std::lock_guard<std::mutex> c(cmu_);
  for (;;) {
    batch_.clear();
    {
      std::lock_guard<std::mutex> q(qmu_);
      if (ops_.empty()) return;
      batch_.swap(ops_);
    }
    for (const Op& op : batch_) {
      switch (op.kind) {
        case Op::kData:
          apply_data(op.blk + op.off, static_cast<size_t>(op.len));
          break;
        case Op::kRelease:
          huge_give(op.blk, cap_);
          held_.fetch_sub(1, std::memory_order_release);
          break;
        case Op::kBegin: apply_chunk_begin(); break;
        case Op::kEnd: apply_chunk_end(op.has_crc, op.crc); break;
        case Op::kResume: apply_resume(); break;
      }
    }
  }
}

void DiscardSink::abort() {
  if (deferred_) reset_ring();
}

SinkResult DiscardSink::finish() {
  if (deferred_ && cur_) {  // the read is over: its last block goes back too
    Op op{Op::kRelease};
    op.blk = cur_;
    push(op);
    cur_ = nullptr;
  }
  drain();
  SinkResult r;
  fold_chunk();
  in_chunk_ = false;
  r.bytes = bytes_;
  r.landed_ns = now_ns();
  r.computed_crc32c = obj_crc_;
  if (host_crc_ && info_.has_crc32c && info_.start_offset == 0 &&
      (info_.size < 0 || static_cast<uint64_t>(info_.size) == bytes_)) {
    any_checked_ = true;
    if (obj_crc_ != info_.crc32c) {
      mismatch_ = true;
      char b[128];
      std::snprintf(b, sizeof(b), "bad CRC on read: got %08x want %08x", obj_crc_, info_.crc32c);
      if (detail_.empty()) detail_ = b;  // keep the first (chunk-level) finding
    }
  }
  r.verified = any_checked_ && !mismatch_;
  r.crc_mismatch = mismatch_;
  r.detail = detail_;
  return r;
}

}  // namespace gcsb
