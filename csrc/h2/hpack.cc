#include "h2/hpack.h"

#include <array>
#include <stdexcept>

namespace gcsb {
namespace {

// RFC 7541 Appendix A static table (1-based).
const std::pair<const char*, const char*> kStatic[61] = {
    {":authority", ""},
    {":method", "GET"},
    {":method", "POST"},
    {":path", "/"},
    {":path", "/index.html"},
    {":scheme", "http"},
    {":scheme", "https"},
    {":status", "200"},
    {":status", "204"},
    {":status", "206"},
    {":status", "304"},
    {":status", "400"},
    {":status", "404"},
    {":status", "500"},
    {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"},
    {"accept-language", ""},
    {"accept-ranges", ""},
    {"accept", ""},
    {"access-control-allow-origin", ""},
    {"age", ""},
    {"allow", ""},
    {"authorization", ""},
    {"cache-control", ""},
    {"content-disposition", ""},
    {"content-encoding", ""},
    {"content-language", ""},
    {"content-length", ""},
    {"content-location", ""},
    {"content-range", ""},
    {"content-type", ""},
    {"cookie", ""},
    {"date", ""},
    {"etag", ""},
    {"expect", ""},
    {"expires", ""},
    {"from", ""},
    {"host", ""},
    {"if-match", ""},
    {"if-modified-since", ""},
    {"if-none-match", ""},
    {"if-range", ""},
    {"if-unmodified-since", ""},
    {"last-modified", ""},
    {"link", ""},
    {"location", ""},
    {"max-forwards", ""},
    {"proxy-authenticate", ""},
    {"proxy-authorization", ""},
    {"range", ""},
    {"referer", ""},
    {"refresh", ""},
    {"retry-after", ""},
    {"server", ""},
    {"set-cookie", ""},
    {"strict-transport-security", ""},
    {"transfer-encoding", ""},
    {"user-agent", ""},
    {"vary", ""},
    {"via", ""},
    {"www-authenticate", ""},
};

// Appendix B as code lengths; codes are canonical (within one length,
// consecutive in symbol order), which reproduces the RFC table exactly.
struct HuffGroup {
  int len;
  std::initializer_list<int> syms;
};
const HuffGroup kHuffGroups[] = {
    {5, {48, 49, 50, 97, 99, 101, 105, 111, 115, 116}},
    {6, {32, 37, 45, 46, 47, 51, 52, 53, 54, 55, 56, 57, 61, 65, 95, 98, 100, 102, 103, 104, 108, 109, 110, 112, 114,
         117}},
    {7, {58, 66, 67, 68, 69, 70, 71, 72, 73, 74, 75, 76, 77, 78, 79, 80, 81, 82, 83, 84, 85, 86, 87, 89, 106, 107, 113,
         118, 119, 120, 121, 122}},
    {8, {38, 42, 44, 59, 88, 90}},
    {10, {33, 34, 40, 41, 63}},
    {11, {39, 43, 124}},
    {12, {35, 62}},
    {13, {0, 36, 64, 91, 93, 126}},
    {14, {94, 125}},
    {15, {60, 96, 123}},
    {19, {92, 195, 208}},
    {20, {128, 130, 131, 162, 184, 194, 224, 226}},
    {21, {153, 161, 167, 172, 176, 177, 179, 209, 216, 217, 227, 229, 230}},
    {22, {129, 132, 133, 134, 136, 146, 154, 156, 160, 163, 164, 169, 170, 173, 178, 181, 185, 186, 187, 189, 190, 196,
          198, 228, 232, 233}},
    {23, {1, 135, 137, 138, 139, 140, 141, 143, 147, 149, 150, 151, 152, 155, 157, 158, 165, 166, 168, 174, 175, 180,
          182, 183, 188, 191, 197, 231, 239}},
    {24, {9, 142, 144, 145, 148, 159, 171, 206, 215, 225, 236, 237}},
    {25, {199, 207, 234, 235}},
    {26, {192, 193, 200, 201, 202, 205, 210, 213, 218, 219, 238, 240, 242, 243, 255}},
    {27, {203, 204, 211, 212, 214, 221, 222, 223, 241, 244, 245, 246, 247, 248, 250, 251, 252, 253, 254}},
    {28, {2, 3, 4, 5, 6, 7, 8, 11, 12, 14, 15, 16, 17, 18, 19, 20, 21, 23, 24, 25, 26, 27, 28, 29, 30, 31, 127, 220,
          249}},
    {30, {10, 13, 22, 256}},
};

struct Huffman {
  uint32_t code[257];
  uint8_t len[257];
  // decoding tree: node -> children; leaf encoded as -(sym+1)
  std::vector<std::array<int, 2>> tree;
  Huffman() {
    uint32_t c = 0;
    int prev = 0;
    int seen = 0;
    for (const auto& g : kHuffGroups) {
      c <<= (g.len - prev);
      prev = g.len;
      std::vector<int> syms(g.syms);
      for (int s : syms) {
        code[s] = c++;
        len[s] = static_cast<uint8_t>(g.len);
        ++seen;
      }
    }
    if (seen != 257) throw std::logic_error("huffman table incomplete");
    tree.push_back({0, 0});
    for (int s = 0; s < 257; ++s) {
      int node = 0;
      for (int b = len[s] - 1; b >= 0; --b) {
        int bit = (code[s] >> b) & 1;
        if (b == 0) {
          tree[node][bit] = -(s + 1);
        } else {
          if (tree[node][bit] == 0) {
            tree.push_back({0, 0});
            tree[node][bit] = static_cast<int>(tree.size() - 1);
          }
          node = tree[node][bit];
        }
      }
    }
  }
};

const Huffman& huff() {
  static Huffman h;
  return h;
}

}  // namespace

size_t huffman_encoded_length(std::string_view s) {
  const Huffman& h = huff();
  uint64_t bits = 0;
  for (unsigned char c : s) bits += h.len[c];
  return static_cast<size_t>((bits + 7) / 8);
}

std::string huffman_encode(std::string_view s) {
  const Huffman& h = huff();
  std::string out;
  uint64_t acc = 0;
  int nbits = 0;
  for (unsigned char c : s) {
    acc = (acc << h.len[c]) | h.code[c];
    nbits += h.len[c];
    while (nbits >= 8) {
      nbits -= 8;
      out.push_back(static_cast<char>((acc >> nbits) & 0xff));
    }
  }
  if (nbits > 0) out.push_back(static_cast<char>(((acc << (8 - nbits)) | ((1u << (8 - nbits)) - 1)) & 0xff));
  return out;
}

bool huffman_decode(const uint8_t* p, size_t n, std::string* out) {
  const Huffman& h = huff();
  int node = 0;
  int depth = 0;      // bits consumed since the last emitted symbol
  bool all_ones = true;
  for (size_t i = 0; i < n; ++i) {
    for (int b = 7; b >= 0; --b) {
      int bit = (p[i] >> b) & 1;
      int nx = h.tree[node][bit];
      ++depth;
      all_ones = all_ones && bit;
      if (nx < 0) {
        int sym = -nx - 1;
        if (sym == 256) return false;  // EOS in the string is an error
        out->push_back(static_cast<char>(sym));
        node = 0;
        depth = 0;
        all_ones = true;
      } else if (nx == 0) {
        return false;
      } else {
        node = nx;
      }
    }
  }
  // padding: strictly fewer than 8 bits, all ones (EOS prefix)
  return depth < 8 && all_ones;
}

void hpack_encode_int(uint64_t v, int prefix_bits, uint8_t flags, std::string* out) {
  const uint64_t maxp = (1u << prefix_bits) - 1;
  if (v < maxp) {
    out->push_back(static_cast<char>(flags | v));
    return;
  }
  out->push_back(static_cast<char>(flags | maxp));
  v -= maxp;
  while (v >= 128) {
    out->push_back(static_cast<char>((v & 127) | 128));
    v >>= 7;
  }
  out->push_back(static_cast<char>(v));
}

bool hpack_decode_int(const uint8_t*& p, const uint8_t* end, int prefix_bits, uint64_t* v) {
  if (p >= end) return false;
  const uint64_t maxp = (1u << prefix_bits) - 1;
  uint64_t x = *p++ & maxp;
  if (x < maxp) {
    *v = x;
    return true;
  }
  int shift = 0;
  for (;;) {
    if (p >= end || shift > 56) return false;
    uint8_t b = *p++;
    x += static_cast<uint64_t>(b & 127) << shift;
    shift += 7;
    if (!(b & 128)) break;
  }
  *v = x;
  return true;
}

static std::string decode_string(const uint8_t*& p, const uint8_t* end) {
  if (p >= end) throw std::runtime_error("hpack: truncated string");
  bool huff_coded = (*p & 0x80) != 0;
  uint64_t len;
  if (!hpack_decode_int(p, end, 7, &len)) throw std::runtime_error("hpack: bad string length");
  if (static_cast<uint64_t>(end - p) < len) throw std::runtime_error("hpack: string overruns block");
  std::string s;
  if (huff_coded) {
    if (!huffman_decode(p, static_cast<size_t>(len), &s)) throw std::runtime_error("hpack: bad huffman string");
  } else {
    s.assign(reinterpret_cast<const char*>(p), static_cast<size_t>(len));
  }
  p += len;
  return s;
}

const std::pair<std::string, std::string>& HpackDecoder::lookup(uint64_t idx) const {
  static thread_local std::pair<std::string, std::string> tmp;
  if (idx == 0) throw std::runtime_error("hpack: index 0");
  if (idx <= 61) {
    tmp.first = kStatic[idx - 1].first;
    tmp.second = kStatic[idx - 1].second;
    return tmp;
  }
  uint64_t d = idx - 62;
  if (d >= table_.size()) throw std::runtime_error("hpack: index out of range");
  return table_[static_cast<size_t>(d)];
}

void HpackDecoder::evict_to(size_t cap) {
  while (size_ > cap && !table_.empty()) {
    size_ -= table_.back().first.size() + table_.back().second.size() + 32;
    table_.pop_back();
  }
}

void HpackDecoder::insert(std::string name, std::string value) {
  size_t sz = name.size() + value.size() + 32;
  if (sz > cap_) {
    evict_to(0);
    return;
  }
  evict_to(cap_ - sz);
  table_.emplace_front(std::move(name), std::move(value));
  size_ += sz;
}

void HpackDecoder::decode(const uint8_t* p, size_t n, HeaderList* out) {
  const uint8_t* end = p + n;
  while (p < end) {
    uint8_t b = *p;
    if (b & 0x80) {  // indexed
      uint64_t idx;
      if (!hpack_decode_int(p, end, 7, &idx)) throw std::runtime_error("hpack: bad index");
      const auto& kv = lookup(idx);
      out->emplace_back(kv.first, kv.second);
    } else if ((b & 0xC0) == 0x40) {  // literal with incremental indexing
      uint64_t idx;
      if (!hpack_decode_int(p, end, 6, &idx)) throw std::runtime_error("hpack: bad index");
      std::string name = idx ? lookup(idx).first : decode_string(p, end);
      std::string value = decode_string(p, end);
      out->emplace_back(name, value);
      insert(std::move(name), std::move(value));
    } else if ((b & 0xE0) == 0x20) {  // dynamic table size update
      uint64_t sz;
      if (!hpack_decode_int(p, end, 5, &sz)) throw std::runtime_error("hpack: bad size update");
      if (sz > max_size_) throw std::runtime_error("hpack: size update above the announced limit");
      cap_ = static_cast<size_t>(sz);
      evict_to(cap_);
    } else {  // literal without indexing (0000) / never indexed (0001)
      uint64_t idx;
      if (!hpack_decode_int(p, end, 4, &idx)) throw std::runtime_error("hpack: bad index");
      std::string name = idx ? lookup(idx).first : decode_string(p, end);
      std::string value = decode_string(p, end);
      out->emplace_back(std::move(name), std::move(value));
    }
  }
}

static void encode_string(std::string_view s, bool huffman, std::string* out) {
  if (huffman) {
    size_t hl = huffman_encoded_length(s);
    if (hl < s.size()) {
      hpack_encode_int(hl, 7, 0x80, out);
      out->append(huffman_encode(s));
      return;
    }
  }
  hpack_encode_int(s.size(), 7, 0x00, out);
  out->append(s.data(), s.size());
}

void HpackEncoder::encode_one(std::string_view name, std::string_view value, std::string* out) const {
  int name_idx = 0;
  for (int i = 0; i < 61; ++i) {
    if (name == kStatic[i].first) {
      if (value == kStatic[i].second) {
        hpack_encode_int(static_cast<uint64_t>(i + 1), 7, 0x80, out);
        return;
      }
      if (!name_idx) name_idx = i + 1;
    }
  }
  // literal header field without indexing (stateless for the peer)
  if (name_idx) {
    hpack_encode_int(static_cast<uint64_t>(name_idx), 4, 0x00, out);
  } else {
    out->push_back(0x00);
    encode_string(name, huffman_, out);
  }
  encode_string(value, huffman_, out);
}

void HpackEncoder::encode(const HeaderList& headers, std::string* out) const {
  for (const auto& kv : headers) encode_one(kv.first, kv.second, out);
}

}  // namespace gcsb
