// Protocol-buffers wire format (encode + zero-copy decode).  No protoc in the
// image, so google.storage.v2 messages are coded by hand (storage_v2.h).
#pragma once
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>

namespace gcsb::pb {

enum WireType : uint32_t { kVarint = 0, kI64 = 1, kLen = 2, kI32 = 5 };

inline void put_varint(std::string* o, uint64_t v) {
  while (v >= 0x80) {
    o->push_back(static_cast<char>((v & 0x7F) | 0x80));
    v >>= 7;
  }
  o->push_back(static_cast<char>(v));
}
inline size_t varint_size(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}
inline void put_tag(std::string* o, uint32_t field, WireType wt) { put_varint(o, (uint64_t(field) << 3) | wt); }
inline void put_int64(std::string* o, uint32_t field, int64_t v) {
  if (v == 0) return;  // proto3 default elided
  put_tag(o, field, kVarint);
  put_varint(o, static_cast<uint64_t>(v));
}
inline void put_int64_always(std::string* o, uint32_t field, int64_t v) {
  put_tag(o, field, kVarint);
  put_varint(o, static_cast<uint64_t>(v));
}
inline void put_bool(std::string* o, uint32_t field, bool v) {
  if (!v) return;
  put_tag(o, field, kVarint);
  o->push_back(1);
}
inline void put_fixed32(std::string* o, uint32_t field, uint32_t v) {
  put_tag(o, field, kI32);
  char b[4];
  std::memcpy(b, &v, 4);  // little-endian host
  o->append(b, 4);
}
inline void put_bytes(std::string* o, uint32_t field, std::string_view v) {
  put_tag(o, field, kLen);
  put_varint(o, v.size());
  o->append(v.data(), v.size());
}
inline void put_string(std::string* o, uint32_t field, std::string_view v) {
  if (v.empty()) return;
  put_bytes(o, field, v);
}
inline void put_message(std::string* o, uint32_t field, const std::string& sub) { put_bytes(o, field, sub); }
// Length-delimited header only (payload written separately, zero-copy).
inline void put_len_header(std::string* o, uint32_t field, uint64_t len) {
  put_tag(o, field, kLen);
  put_varint(o, len);
}

class Reader {
 public:
  Reader(const void* p, size_t n) : p_(static_cast<const uint8_t*>(p)), end_(p_ + n) {}
  explicit Reader(std::string_view s) : Reader(s.data(), s.size()) {}
  bool done() const { return p_ >= end_; }
  bool ok() const { return ok_; }
  // Reads the next tag; false at end or on error.
  bool next(uint32_t* field, WireType* wt) {
    if (p_ >= end_ || !ok_) return false;
    uint64_t t = varint();
    if (!ok_) return false;
    *field = static_cast<uint32_t>(t >> 3);
    *wt = static_cast<WireType>(t & 7);
    return *field != 0;
  }
  uint64_t varint() {
    uint64_t v = 0;
    int s = 0;
    while (p_ < end_ && s < 64) {
      uint8_t b = *p_++;
      v |= uint64_t(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
      s += 7;
    }
    ok_ = false;
    return 0;
  }
  uint32_t fixed32() {
    if (end_ - p_ < 4) {
      ok_ = false;
      return 0;
    }
    uint32_t v;
    std::memcpy(&v, p_, 4);
    p_ += 4;
    return v;
  }
  uint64_t fixed64() {
    if (end_ - p_ < 8) {
      ok_ = false;
      return 0;
    }
    uint64_t v;
    std::memcpy(&v, p_, 8);
    p_ += 8;
    return v;
  }
  std::string_view bytes() {
    uint64_t n = varint();
    if (!ok_ || static_cast<uint64_t>(end_ - p_) < n) {
      ok_ = false;
      return {};
    }
    std::string_view s(reinterpret_cast<const char*>(p_), static_cast<size_t>(n));
    p_ += n;
    return s;
  }
  void skip(WireType wt) {
    switch (wt) {
      case kVarint: varint(); break;
      case kI64: fixed64(); break;
      case kLen: bytes(); break;
      case kI32: fixed32(); break;
      default: ok_ = false;
    }
  }

 private:
  const uint8_t* p_;
  const uint8_t* end_;
  bool ok_ = true;
};

}  // namespace gcsb::pb
