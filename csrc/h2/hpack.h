// HPACK (RFC 7541) header compression for the native HTTP/2 stack.
//
// Reference: grpc-go speaks HTTP/2 to storage.googleapis.com for the gRPC
// client (reference main.go:106-117, go.mod:20).  No gRPC C++ library or
// nghttp2 exists in this image, so the framing and header coding are
// implemented here.  The decoder handles the full spec (static + dynamic
// table, size updates, Huffman strings) so it interoperates with grpc-core
// peers; the encoder emits literal-without-indexing / static-indexed fields
// (stateless, always valid) with optional Huffman coding.
#pragma once
#include <cstdint>
#include <deque>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace gcsb {

using HeaderList = std::vector<std::pair<std::string, std::string>>;

class HpackDecoder {
 public:
  explicit HpackDecoder(uint32_t max_table_size = 4096) : max_size_(max_table_size), cap_(max_table_size) {}
  // Decodes a complete header block; throws std::runtime_error on errors.
  void decode(const uint8_t* p, size_t n, HeaderList* out);
  void set_max_table_size(uint32_t s) { max_size_ = s; }
  size_t table_size() const { return size_; }
  size_t table_entries() const { return table_.size(); }

 private:
  const std::pair<std::string, std::string>& lookup(uint64_t idx) const;
  void insert(std::string name, std::string value);
  void evict_to(size_t cap);
  uint32_t max_size_;  // limit announced in our SETTINGS
  size_t cap_;         // current dynamic table capacity
  size_t size_ = 0;
  std::deque<std::pair<std::string, std::string>> table_;  // front = newest
};

class HpackEncoder {
 public:
  explicit HpackEncoder(bool huffman = false) : huffman_(huffman) {}
  void encode(const HeaderList& headers, std::string* out) const;
  void encode_one(std::string_view name, std::string_view value, std::string* out) const;

 private:
  bool huffman_;
};

// Huffman coding (RFC 7541 Appendix B canonical code).
std::string huffman_encode(std::string_view s);
bool huffman_decode(const uint8_t* p, size_t n, std::string* out);
size_t huffman_encoded_length(std::string_view s);

// Integer representation with an N-bit prefix.
void hpack_encode_int(uint64_t v, int prefix_bits, uint8_t first_byte_flags, std::string* out);
bool hpack_decode_int(const uint8_t*& p, const uint8_t* end, int prefix_bits, uint64_t* v);

}  // namespace gcsb
