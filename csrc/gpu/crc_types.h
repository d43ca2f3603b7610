// Plain-data types shared by the CRC32C kernels, their launchers and the
// host-side emulator (crc_host.cc) that checks the kernel algorithm on CPU.
#pragma once
#include <cstdint>

namespace gcsb {

// Tile geometry: a wave64 owns one tile of R rounds x 4 KiB; in each round
// lane l reads its own contiguous 64-byte chunk (kCrcChunkPieces x 16 B) at
// round_base + 64 l, so every 128-byte line is consumed by 2 lanes within 4
// consecutive load instructions (L1-friendly), and a lane's CRC chain is
// contiguous inside a chunk.  Between its chunks a lane's state is shifted
// over the 4032-byte gap (one 4-lookup shift), and the 64 lane states fold in
// a 6-level wave tree (shifts of 64 B * 2^lv).
//   R = 4 (16 KiB tiles): 16 + 0.75 + 1.5 LDS lookups per 16 B; bulk rate.
//   R = 1 (4 KiB tiles) : 16 + 6 lookups per 16 B, but 4x the waves: a 2 MiB
//                         ring slot becomes 512 waves instead of 128, so a
//                         latency-bound slot-sized batch spreads over the chip.
constexpr int kCrcChunkPieces = 4;
constexpr int kCrcChunkBytes = 16 * kCrcChunkPieces;  // 64 B per lane per round
constexpr int kCrcRoundBytes = 64 * kCrcChunkBytes;   // 4 KiB per round
constexpr int kCrcLaneGap = kCrcRoundBytes - kCrcChunkBytes;  // 4032 B between a lane's chunks
constexpr int kCrcMinTileLog2 = 12;                   // 4 KiB tiles (R = 1)
constexpr int kCrcMaxTileLog2 = 14;                   // 16 KiB tiles (R = 4)
constexpr int kCrcMinTile = 1 << kCrcMinTileLog2;     // sizing tile scratch: the most tiles a batch can have
constexpr int kCrcTileShiftLevels = 13;               // tile_shift[s] = shift by 4 KiB * 2^s, s = 0..12
// Batches whose segments all fold within kCrcFusedMaxTiles tiles use ONE
// launch: the last workgroup to finish its tiles folds every segment (one wave
// per segment) -- ring slots always qualify.  Longer segments (bulk
// gpu_crc32c) get a separate fold kernel with 8 waves per segment.
constexpr uint32_t kCrcFusedMaxTiles = 64 * 16;  // <= 16 Horner steps per lane (2 prefetch rounds)
constexpr int kMaxSeg = 32;
// Tile scratch layout: word 0 = the fused kernel's "workgroups done" counter
// (zero between launches), tiles from word kCrcScratchHeader.
constexpr int kCrcScratchHeader = 64;

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
  uint32_t tile_log2;  // 12 or 14, chosen by finalize_crc_batch
  uint32_t max_seg_tiles;
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
  uint32_t tile_shift[kCrcTileShiftLevels][4][256];  // shift by 4 KiB * 2^s
};

// Number of tiles (of 2^tile_log2 bytes) covering a segment's 16-byte pieces
// except its last one, which the fold adds as the 1..16-byte tail.
inline void crc_segment_geometry(uintptr_t addr, uint32_t len, uint32_t tile_log2, uint32_t* ntiles) {
  if (len == 0) {
    *ntiles = 0;
    return;
  }
  uintptr_t a16 = addr & ~uintptr_t(15);
  uint64_t pieces = (addr + len - a16 + 15) / 16;
  uint64_t full = pieces - 1;
  const uint64_t per_tile = (uint64_t(1) << tile_log2) / 16;
  *ntiles = static_cast<uint32_t>((full + per_tile - 1) / per_tile);
}

void build_crc_tables(CrcTables* t);
// Fills seg.tile_base/ntiles/fixup, batch.total_tiles/max_seg_tiles and picks
// the tile size: 4 KiB tiles for batches up to 4 MiB (slot-sized, latency
// bound), 16 KiB above (bulk).  tile_log2 != 0 forces a size (tests, A/B);
// GCSB_CRC_TILE=4k|16k overrides the automatic choice.
void finalize_crc_batch(CrcBatch* b, uint32_t tile_log2 = 0);
// Words of tile scratch (header + tiles) a batch of up to `tiles` tiles needs.
inline uint64_t crc_scratch_words(uint64_t tiles) { return tiles + kCrcScratchHeader; }
// Host emulation of the kernels' math (same tables, same tile/lane/fold
// decomposition): the CPU test oracle.  fold_waves = 1 mirrors the fused
// epilogue, 8 the separate fold kernel.
CrcSegResult emulate_crc32c_segment(const uint8_t* addr, uint32_t len, const CrcTables& t, uint32_t expected,
                                    bool check, uint32_t tile_log2 = kCrcMaxTileLog2, int fold_waves = 8);

}  // namespace gcsb
