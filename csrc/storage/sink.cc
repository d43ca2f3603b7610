#include "storage/sink.h"

#include <cstdio>
#include <cstdlib>

#include "core/crc32c.h"
#include "core/util.h"

namespace gcsb {

DiscardSink::DiscardSink(size_t chunk_bytes, bool host_crc)
    : buf_(static_cast<uint8_t*>(std::aligned_alloc(4096, (chunk_bytes + 4095) / 4096 * 4096))),
      cap_(chunk_bytes),
      host_crc_(host_crc) {}

DiscardSink::~DiscardSink() { std::free(buf_); }

void DiscardSink::begin(const ObjectInfo& info) {
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
  return Window{buf_, cap_};
}

void DiscardSink::commit(size_t n) {
  // each byte is CRC'd once: inside a chunk into the chunk CRC (combined
  // into the object CRC at chunk end), outside directly into the object CRC
  if (host_crc_) {
    if (in_chunk_) {
      chunk_crc_ = crc32c_extend(chunk_crc_, buf_, n);
      chunk_len_ += n;
    } else {
      obj_crc_ = crc32c_extend(obj_crc_, buf_, n);
    }
  }
  bytes_ += n;
}

void DiscardSink::fold_chunk() {
  if (in_chunk_ && chunk_len_) obj_crc_ = crc32c_combine(obj_crc_, chunk_crc_, chunk_len_);
  chunk_crc_ = 0;
  chunk_len_ = 0;
}

void DiscardSink::chunk_begin(size_t) {
  fold_chunk();
  in_chunk_ = true;
}

void DiscardSink::chunk_end(bool has_crc, uint32_t crc) {
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
  // bytes of the interrupted chunk stay counted in the object CRC; the chunk
  // itself can no longer be checked on its own.
  (void)offset;
  if (in_chunk_) chunk_partial_ = true;
  fold_chunk();
  in_chunk_ = false;
}

SinkResult DiscardSink::finish() {
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
