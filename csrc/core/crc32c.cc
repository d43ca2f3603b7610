// Host CRC32C: SSE4.2 three-stream interleave + table fallback + GF(2) algebra.
// See crc32c.h for the raw/shift/fixup vocabulary.
#include "core/crc32c.h"

#include <cstring>
#include <mutex>
#include <nmmintrin.h>

namespace gcsb {
namespace {

struct Tables {
  uint32_t slice[8][256];
  uint32_t x2n[64];  // x^(2^k) mod P
  // shift tables for the interleaved hardware path
  uint32_t shift_blk[4][256];   // shift by kBlk bytes
  uint32_t shift_2blk[4][256];  // shift by 2*kBlk bytes
};

constexpr size_t kBlk = 8192;  // bytes per lane of the 3-way interleave

// GF(2) polynomial product mod P and x^(2^k) powers: the standard CRC
// combine algebra, structured after zlib's multmodp()/x2nmodp() (crc32.c,
// zlib licence, Mark Adler), here for the Castagnoli polynomial.
uint32_t multmodp_impl(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ kCrc32cPoly : b >> 1;
  }
  return p;
}

const Tables& tables() {
  static Tables* t = [] {
    auto* tb = new Tables();
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t c = b;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrc32cPoly : c >> 1;
      tb->slice[0][b] = c;
    }
    for (uint32_t b = 0; b < 256; ++b)
      for (int k = 1; k < 8; ++k) {
        uint32_t c = tb->slice[k - 1][b];
        tb->slice[k][b] = (c >> 8) ^ tb->slice[0][c & 0xff];
      }
    uint32_t p = 1u << 30;  // x^1
    for (int k = 0; k < 64; ++k) {
      tb->x2n[k] = p;
      p = multmodp_impl(p, p);
    }
    return tb;
  }();
  return *t;
}

uint32_t x2nmodp(uint64_t n, unsigned k) {
  const Tables& t = tables();
  uint32_t p = 1u << 31;  // x^0
  while (n) {
    if (n & 1) p = multmodp_impl(t.x2n[k & 63], p);
    n >>= 1;
    ++k;
  }
  return p;
}

const Tables& tables_with_shift() {
  static std::once_flag once;
  static Tables* tb = const_cast<Tables*>(&tables());
  std::call_once(once, [] {
    crc32c_build_shift_table(kBlk, tb->shift_blk);
    crc32c_build_shift_table(2 * kBlk, tb->shift_2blk);
  });
  return *tb;
}

uint32_t raw_update_sw(uint32_t s, const uint8_t* p, size_t n) {
  const Tables& t = tables();
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    s = (s >> 8) ^ t.slice[0][(s ^ *p++) & 0xff];
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    uint32_t lo = static_cast<uint32_t>(v) ^ s;
    uint32_t hi = static_cast<uint32_t>(v >> 32);
    s = t.slice[7][lo & 0xff] ^ t.slice[6][(lo >> 8) & 0xff] ^ t.slice[5][(lo >> 16) & 0xff] ^
        t.slice[4][lo >> 24] ^ t.slice[3][hi & 0xff] ^ t.slice[2][(hi >> 8) & 0xff] ^
        t.slice[1][(hi >> 16) & 0xff] ^ t.slice[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) s = (s >> 8) ^ t.slice[0][(s ^ *p++) & 0xff];
  return s;
}

__attribute__((target("sse4.2"))) uint32_t raw_update_hw1(uint32_t s, const uint8_t* p, size_t n) {
  uint64_t c = s;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = _mm_crc32_u8(static_cast<uint32_t>(c), *p++);
    --n;
  }
  while (n >= 32) {
    uint64_t a, b, d, e;
    std::memcpy(&a, p, 8);
    std::memcpy(&b, p + 8, 8);
    std::memcpy(&d, p + 16, 8);
    std::memcpy(&e, p + 24, 8);
    c = _mm_crc32_u64(c, a);
    c = _mm_crc32_u64(c, b);
    c = _mm_crc32_u64(c, d);
    c = _mm_crc32_u64(c, e);
    p += 32;
    n -= 32;
  }
  while (n >= 8) {
    uint64_t a;
    std::memcpy(&a, p, 8);
    c = _mm_crc32_u64(c, a);
    p += 8;
    n -= 8;
  }
  while (n--) c = _mm_crc32_u8(static_cast<uint32_t>(c), *p++);
  return static_cast<uint32_t>(c);
}

// Three independent dependency chains hide the 3-cycle latency of `crc32`.
__attribute__((target("sse4.2"))) uint32_t raw_update_hw(uint32_t s, const uint8_t* p, size_t n) {
  if (n < 3 * kBlk) return raw_update_hw1(s, p, n);
  const Tables& t = tables_with_shift();
  while (n >= 3 * kBlk) {
    uint64_t c0 = s, c1 = 0, c2 = 0;
    const uint8_t* p0 = p;
    const uint8_t* p1 = p + kBlk;
    const uint8_t* p2 = p + 2 * kBlk;
    for (size_t i = 0; i < kBlk; i += 8) {
      uint64_t a, b, d;
      std::memcpy(&a, p0 + i, 8);
      std::memcpy(&b, p1 + i, 8);
      std::memcpy(&d, p2 + i, 8);
      c0 = _mm_crc32_u64(c0, a);
      c1 = _mm_crc32_u64(c1, b);
      c2 = _mm_crc32_u64(c2, d);
    }
    s = crc32c_apply_shift_table(t.shift_2blk, static_cast<uint32_t>(c0)) ^
        crc32c_apply_shift_table(t.shift_blk, static_cast<uint32_t>(c1)) ^ static_cast<uint32_t>(c2);
    p += 3 * kBlk;
    n -= 3 * kBlk;
  }
  return raw_update_hw1(s, p, n);
}

bool detect_hw() { return __builtin_cpu_supports("sse4.2"); }

}  // namespace

bool crc32c_hw_available() {
  static bool hw = detect_hw();
  return hw;
}

uint32_t crc32c_raw_update(uint32_t state, const void* data, size_t n) {
  const auto* p = static_cast<const uint8_t*>(data);
  return crc32c_hw_available() ? raw_update_hw(state, p, n) : raw_update_sw(state, p, n);
}

uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  return ~crc32c_raw_update(~crc, data, n);
}

uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }

uint32_t gf2_multmodp(uint32_t a, uint32_t b) { return multmodp_impl(a, b); }

uint32_t crc32c_x8n(uint64_t nbytes) { return x2nmodp(nbytes, 3); }

uint32_t crc32c_shift(uint32_t state, uint64_t nbytes) {
  if (nbytes == 0 || state == 0) return state;
  return multmodp_impl(crc32c_x8n(nbytes), state);
}

uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return crc32c_shift(crc_a, len_b) ^ crc_b;
}

uint32_t crc32c_fixup(uint64_t nbytes) { return crc32c_shift(0xFFFFFFFFu, nbytes) ^ 0xFFFFFFFFu; }

void crc32c_build_slice16(uint32_t slice[16][256]) {
  const Tables& t = tables();
  for (int b = 0; b < 256; ++b) slice[0][b] = t.slice[0][b];
  for (int k = 1; k < 16; ++k)
    for (int b = 0; b < 256; ++b) {
      uint32_t c = slice[k - 1][b];
      slice[k][b] = (c >> 8) ^ t.slice[0][c & 0xff];
    }
}

void crc32c_build_shift_table(uint64_t nbytes, uint32_t tab[4][256]) {
  const uint32_t op = crc32c_x8n(nbytes);
  for (int j = 0; j < 4; ++j)
    for (uint32_t b = 0; b < 256; ++b) tab[j][b] = multmodp_impl(op, b << (8 * j));
}

uint32_t crc32c_apply_shift_table(const uint32_t tab[4][256], uint32_t s) {
  return tab[0][s & 0xff] ^ tab[1][(s >> 8) & 0xff] ^ tab[2][(s >> 16) & 0xff] ^ tab[3][s >> 24];
}

}  // namespace gcsb
