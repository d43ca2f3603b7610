#include "storage/host_arena.h"

#include <cstring>
#include <stdexcept>

#include "core/crc32c.h"
#include "core/util.h"

namespace gcsb {

HostArena::HostArena(size_t slot_bytes, int slots)
    : slot_bytes_(slot_bytes < 4096 ? 4096 : slot_bytes), slots_(slots < 2 ? 2 : slots) {
  mem_.resize(slot_bytes_ * static_cast<size_t>(slots_));
}

std::pair<uint8_t*, size_t> HostArena::recv_window() {
  if (cur_ < 0 || used_ == slot_bytes_) {
    // the sink copied every payload run out at commit: a slot is free as
    // soon as the reader leaves it
    cur_ = (cur_ + 1) % slots_;
    used_ = 0;
  }
  return {mem_.data() + slot_bytes_ * static_cast<size_t>(cur_) + used_, slot_bytes_ - used_};
}

void HostArena::received(size_t n) {
  used_ += n;
  ++recvs_;
  bytes_ += n;
}

bool HostArena::contains(const uint8_t* p, size_t n) const {
  if (cur_ < 0) return false;
  const uint8_t* base = mem_.data() + slot_bytes_ * static_cast<size_t>(cur_);
  return p >= base && p + n <= base + used_;
}

void InplaceHostSink::begin(const ObjectInfo& info) {
  info_ = info;
  data_.clear();
  if (info.size > 0) data_.reserve(static_cast<size_t>(info.size));
  in_chunk_ = chunk_broken_ = mismatch_ = false;
  chunk_crc_ = 0;
  chunk_len_ = 0;
  detail_.clear();
}

void InplaceHostSink::update_info(const ObjectInfo& info) {
  if (info.has_crc32c) {
    info_.has_crc32c = true;
    info_.crc32c = info.crc32c;
  }
  if (info.size >= 0) info_.size = info.size;
}

Window InplaceHostSink::acquire(size_t want) {
  window_.resize(want ? want : 1);
  return Window{window_.data(), window_.size()};
}

void InplaceHostSink::commit(size_t n) { land(window_.data(), n); }

void InplaceHostSink::commit_inplace(const uint8_t* p, size_t n) {
  if (!arena_->contains(p, n)) throw std::logic_error("InplaceHostSink: bytes outside the arena's current slot");
  ++inplace_;
  land(p, n);
}

void InplaceHostSink::land(const uint8_t* p, size_t n) {
  data_.insert(data_.end(), p, p + n);
  if (in_chunk_) {
    chunk_crc_ = crc32c_extend(chunk_crc_, p, n);
    chunk_len_ += n;
  }
}

void InplaceHostSink::chunk_begin(size_t) {
  in_chunk_ = true;
  chunk_broken_ = false;
  chunk_crc_ = 0;
  chunk_len_ = 0;
}

void InplaceHostSink::chunk_end(bool has_crc, uint32_t crc) {
  if (!in_chunk_) return;
  in_chunk_ = false;
  if (has_crc && !chunk_broken_) {
    ++chunks_checked_;
    if (chunk_crc_ != crc) {
      mismatch_ = true;
      detail_ = "chunk crc32c mismatch at offset " + std::to_string(data_.size() - chunk_len_);
    }
  }
}

void InplaceHostSink::resume_at(int64_t) {
  if (in_chunk_) chunk_broken_ = true;
}

SinkResult InplaceHostSink::finish() {
  SinkResult r;
  r.bytes = data_.size();
  r.landed_ns = now_ns();
  r.computed_crc32c = crc32c_extend(0, data_.data(), data_.size());
  r.crc_mismatch = mismatch_;
  r.detail = detail_;
  if (info_.has_crc32c && info_.start_offset == 0 && info_.size >= 0 &&
      static_cast<uint64_t>(info_.size) == data_.size()) {
    if (r.computed_crc32c != info_.crc32c) {
      r.crc_mismatch = true;
      r.detail = "object crc32c mismatch";
    }
    r.verified = !r.crc_mismatch;
  }
  return r;
}

}  // namespace gcsb
