// Plain-data types shared by the CRC32C kernels, their launchers and the
// host-side emulator (crc_emul.cc) that checks the kernel algorithm on CPU.
#pragma once
#include <cstdint>

namespace gcsb {

// K1 geometry: a wave64 owns one 16 KiB tile, read in kCrcRounds rounds of
// 4 KiB; in each round lane l reads its own contiguous 64-byte chunk
// (kCrcChunkPieces x 16 B) at round_base + 64 l, so every 128-byte line is
// consumed by 2 lanes within 4 consecutive load instructions (L1-friendly),
// and a lane's CRC chain is contiguous inside a chunk.  Between its chunks a
// lane's state is shifted over the 4032-byte gap (one 4-lookup shift), and the
// 64 lane states fold in a 6-level wave tree (shifts of 64 B * 2^lv).  LDS
// lookups per 16 B: 16 (slice-by-16) + 0.75 (gaps) + 1.5 (tree).
constexpr int kCrcChunkPieces = 4;
constexpr int kCrcChunkBytes = 16 * kCrcChunkPieces;  // 64 B per lane per round
constexpr int kCrcRoundBytes = 64 * kCrcChunkBytes;   // 4 KiB per round
constexpr int kCrcRounds = 4;
constexpr int kCrcTile = kCrcRounds * kCrcRoundBytes;  // 16 KiB per wave
constexpr int kCrcLaneGap = kCrcRoundBytes - kCrcChunkBytes;  // 4032 B between a lane's chunks
constexpr int kMaxSeg = 32;

struct CrcSeg {
  const uint8_t* addr;
  uint32_t len;
  uint32_t tile_base;  // first tile index in the batch's tile scratch
  uint32_t ntiles;
  uint32_t expected;
  uint32_t fixup;      // crc32c(d) = raw(d) ^ fixup(|d|)
  uint32_t flags;      // bit0: compare against expected
};

struct CrcBatch {
  uint32_t nseg;
  uint32_t total_tiles;
  CrcSeg seg[kMaxSeg];
};

struct CrcSegResult {
  uint32_t raw;
  uint32_t crc;
  uint32_t status;  // 0 not checked, 1 match, 2 mismatch
  uint32_t pad;
};

struct CrcTables {
  uint32_t slice16[16][256];
  uint32_t lane_shift[7][4][256];  // [0..5]: shift by kCrcChunkBytes * 2^lv (wave tree); [6]: kCrcLaneGap
  uint32_t tile_shift[9][4][256];  // shift by kCrcTile * 2^s, s = 0..8 (last = 256 tiles)
  // slice-by-16 split into nibble tables: byte p of a 16-byte block (table
  // slice16[15-p]) = nib[2p][lo nibble] ^ nib[2p+1][hi nibble] (GF(2)-linear)
  uint32_t nib[32][16];
};

// Number of kCrcTile tiles covering a segment's full 16-byte pieces (host helper).
inline void crc_segment_geometry(uintptr_t addr, uint32_t len, uint32_t* ntiles) {
  if (len == 0) {
    *ntiles = 0;
    return;
  }
  uintptr_t a16 = addr & ~uintptr_t(15);
  uint64_t pieces = (addr + len - a16 + 15) / 16;
  uint64_t full = pieces - 1;
  constexpr uint64_t per_tile = kCrcTile / 16;
  *ntiles = static_cast<uint32_t>((full + per_tile - 1) / per_tile);
}

// Host emulation of K1+K2 (same tables, same tile/lane decomposition) — the
// CPU test oracle for the kernel math.
void build_crc_tables(CrcTables* t);
// Fills seg.tile_base/ntiles/fixup and batch.total_tiles.
void finalize_crc_batch(CrcBatch* b);
CrcSegResult emulate_crc32c_segment(const uint8_t* addr, uint32_t len, const CrcTables& t, uint32_t expected,
                                    bool check);

}  // namespace gcsb
