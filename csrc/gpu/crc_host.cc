// Host half of the GPU CRC32C engine: table construction, batch geometry and a
// bit-exact emulator of kernels K1/K2 (the CPU-side oracle for their math).
#include <cstdlib>
#include <cstring>
#include <vector>

#include "core/crc32c.h"
#include "gpu/crc_types.h"

namespace gcsb {

void build_crc_tables(CrcTables* t) {
  crc32c_build_slice16(t->slice16);
  for (int lv = 0; lv < 6; ++lv) crc32c_build_shift_table(static_cast<uint64_t>(kCrcChunkBytes) << lv, t->lane_shift[lv]);
  crc32c_build_shift_table(kCrcLaneGap, t->lane_shift[6]);
  for (int lv = 0; lv < kCrcTileShiftLevels; ++lv)
    crc32c_build_shift_table(static_cast<uint64_t>(kCrcRoundBytes) << lv, t->tile_shift[lv]);
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 32; ++i)
      t->lane_k[l][i] = crc32c_shift(1u << i, static_cast<uint64_t>(kCrcChunkBytes) * (63 - l));
  for (uint32_t d = 0; d < kCrcFusedMaxTiles; ++d) {
    // column i of shift by d tiles = shift of column i by one tile, d times
    for (int i = 0; i < 32; ++i)
      t->tile_k[d][i] = d == 0 ? (1u << i) : crc32c_shift(t->tile_k[d - 1][i], kCrcMinTile);
  }
}

namespace {
uint32_t auto_tile_log2(uint64_t total_bytes) {
  return total_bytes <= (4u << 20) ? kCrcMinTileLog2 : kCrcMaxTileLog2;
}
}  // namespace

void finalize_crc_batch(CrcBatch* b, uint32_t tile_log2) {
  uint64_t bytes = 0;
  for (uint32_t i = 0; i < b->nseg; ++i) bytes += b->seg[i].len;
  b->tile_log2 = tile_log2 ? tile_log2 : auto_tile_log2(bytes);
  uint32_t tiles = 0, mx = 0;
  for (uint32_t i = 0; i < b->nseg; ++i) {
    CrcSeg& s = b->seg[i];
    s.tile_base = tiles;
    crc_segment_geometry(reinterpret_cast<uintptr_t>(s.addr), s.len, b->tile_log2, &s.ntiles);
    s.fixup = crc32c_fixup(s.len);
    tiles += s.ntiles;
    if (s.ntiles > mx) mx = s.ntiles;
  }
  b->total_tiles = tiles;
  b->max_seg_tiles = mx;
}

namespace {
uint32_t shift4(const uint32_t tab[4][256], uint32_t s) { return crc32c_apply_shift_table(tab, s); }
uint32_t update16(const uint32_t sl[16][256], uint32_t state, const uint32_t v[4]) {
  const uint32_t x = state ^ v[0];
  uint32_t c = sl[15][x & 0xff] ^ sl[14][(x >> 8) & 0xff] ^ sl[13][(x >> 16) & 0xff] ^ sl[12][x >> 24];
  c ^= sl[11][v[1] & 0xff] ^ sl[10][(v[1] >> 8) & 0xff] ^ sl[9][(v[1] >> 16) & 0xff] ^ sl[8][v[1] >> 24];
  c ^= sl[7][v[2] & 0xff] ^ sl[6][(v[2] >> 8) & 0xff] ^ sl[5][(v[2] >> 16) & 0xff] ^ sl[4][v[2] >> 24];
  c ^= sl[3][v[3] & 0xff] ^ sl[2][(v[3] >> 8) & 0xff] ^ sl[1][(v[3] >> 16) & 0xff] ^ sl[0][v[3] >> 24];
  return c;
}
uint32_t mask_low_bytes(uint32_t w, int keep_from) {
  if (keep_from <= 0) return w;
  if (keep_from >= 4) return 0;
  return w & (0xFFFFFFFFu << (8 * keep_from));
}
}  // namespace

CrcSegResult emulate_crc32c_segment(const uint8_t* addr_p, uint32_t len, const CrcTables& t, uint32_t expected,
                                    bool check, uint32_t tile_log2, int fold_waves) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(addr_p);
  const int rounds = 1 << (tile_log2 - kCrcMinTileLog2);
  const intptr_t tile_bytes = intptr_t(1) << tile_log2;
  const int lvl0 = static_cast<int>(tile_log2) - kCrcMinTileLog2;  // tile_shift index of a 1-tile shift
  uint32_t T = 0;
  crc_segment_geometry(addr, len, tile_log2, &T);
  std::vector<uint32_t> tiles(T);
  const bool slot = fold_waves == 0;
  if (slot && (tile_log2 != static_cast<uint32_t>(kCrcMinTileLog2) || T > kCrcFusedMaxTiles)) {
    CrcSegResult bad{};
    bad.status = 3;  // outside the slot kernel's domain
    return bad;
  }
  uint32_t slot_acc = 0;
  // tile kernel: per-lane chains over R rounds, 6-level wave tree
  for (uint32_t tt = 0; tt < T; ++tt) {
    const uintptr_t a16 = addr & ~uintptr_t(15);
    const uint64_t full = (addr + len - a16 + 15) / 16 - 1;
    const intptr_t vend = static_cast<intptr_t>(a16 + 16 * full);
    const intptr_t tstart = vend - tile_bytes * static_cast<intptr_t>(T - tt);
    uint32_t lanes[64];
    for (int lane = 0; lane < 64; ++lane) {
      uint32_t state = 0;
      for (int k = 0; k < rounds; ++k) {
        if (k) state = shift4(t.lane_shift[6], state);
        for (int j = 0; j < kCrcChunkPieces; ++j) {
          const intptr_t p = tstart + static_cast<intptr_t>(kCrcRoundBytes) * k +
                             static_cast<intptr_t>(kCrcChunkBytes) * lane + 16 * j;
          uint32_t v[4] = {0, 0, 0, 0};
          if (p + 16 > static_cast<intptr_t>(addr)) std::memcpy(v, reinterpret_cast<const void*>(p), 16);
          if (p < static_cast<intptr_t>(addr) && p + 16 > static_cast<intptr_t>(addr)) {
            const int h = static_cast<int>(static_cast<intptr_t>(addr) - p);
            v[0] = mask_low_bytes(v[0], h);
            v[1] = mask_low_bytes(v[1], h - 4);
            v[2] = mask_low_bytes(v[2], h - 8);
            v[3] = mask_low_bytes(v[3], h - 12);
          }
          state = update16(t.slice16, state, v);
        }
      }
      lanes[lane] = state;
    }
    if (slot) {
      // slot kernel: lane -> tile end (lane_k), tile -> segment end (tile_k)
      uint32_t c = 0;
      for (int lane = 0; lane < 64; ++lane) c ^= crc_apply_columns(t.lane_k[lane], lanes[lane]);
      slot_acc ^= crc_apply_columns(t.tile_k[T - 1 - tt], c);
      continue;
    }
    for (int lv = 0; lv < 6; ++lv) {
      uint32_t nxt[64];
      for (int lane = 0; lane < 64; ++lane) {
        uint32_t other = lane + (1 << lv) < 64 ? lanes[lane + (1 << lv)] : lanes[lane];
        uint32_t shifted = shift4(t.lane_shift[lv], lanes[lane]);
        nxt[lane] = ((lane & ((2 << lv) - 1)) == 0) ? (shifted ^ other) : lanes[lane];
      }
      std::memcpy(lanes, nxt, sizeof(lanes));
    }
    tiles[tt] = lanes[0];
  }
  // fold: W waves, thread k folds tiles T-1-(k + S m) by Horner with stride
  // S = 64 W tiles, then a tree over the 64 W threads (shift 2^lv tiles)
  const int W = slot ? 1 : fold_waves;
  int logw = 0;
  while ((1 << logw) < W) ++logw;
  const int S = 64 * W;
  std::vector<uint32_t> acc(static_cast<size_t>(S));
  const int M = static_cast<int>((T + S - 1) / S);
  for (int k = 0; k < S; ++k) {
    uint32_t a = 0;
    for (int m = M - 1; m >= 0; --m) {
      a = shift4(t.tile_shift[lvl0 + 6 + logw], a);
      uint32_t j = static_cast<uint32_t>(k) + static_cast<uint32_t>(S) * static_cast<uint32_t>(m);
      if (j < T) a ^= tiles[T - 1 - j];
    }
    acc[static_cast<size_t>(k)] = a;
  }
  for (int lv = 0; lv < 6 + logw; ++lv)
    for (int k = 0; k < S; k += (2 << lv)) acc[k] ^= shift4(t.tile_shift[lvl0 + lv], acc[k + (1 << lv)]);
  uint32_t raw = slot ? slot_acc : acc[0];
  // tail: the last 1..16 bytes, slice-by-r with one independent lookup per byte
  if (len > 0) {
    const uintptr_t a16 = addr & ~uintptr_t(15);
    const uintptr_t e = addr + len;
    const uintptr_t vend = a16 + 16 * ((e - a16 + 15) / 16 - 1);
    const uintptr_t p0 = vend > addr ? vend : addr;
    const int r = static_cast<int>(e - p0);
    uint32_t x = 0;
    for (int i = 0; i < r; ++i) {
      const uint32_t sb = i < 4 ? (raw >> (8 * i)) & 0xff : 0;
      x ^= t.slice16[r - 1 - i][(*reinterpret_cast<const uint8_t*>(p0 + i) ^ sb) & 0xff];
    }
    raw = x ^ (r < 4 ? raw >> (8 * r) : 0u);
  }
  CrcSegResult res;
  res.raw = raw;
  res.crc = raw ^ crc32c_fixup(len);
  res.status = check ? (res.crc == expected ? 1u : 2u) : 0u;
  res.pad = 0;
  return res;
}

}  // namespace gcsb
