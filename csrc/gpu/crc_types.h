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
// Tile scratch layout: word 0 = the fused kernels' "workgroups done" counter
// (the slot kernel's root counter), then kCrcCounterGroups group counters of
// the slot kernel kCrcCounterStride words apart (all zero between launches),
// tiles from word kCrcScratchHeader.  Same-address device-scope atomics
// serialise at ~14 ns each on MI355X (profiles/r2_crc_slot): 256 workgroups
// on one counter cost 3.6 us, split over 16 lines 0.4 us.
constexpr int kCrcCounterGroups = 16;
constexpr int kCrcCounterStride = 1024;  // 4 KiB apart: different memory channels
constexpr int kCrcScratchHeader = kCrcCounterStride * (kCrcCounterGroups + 1);

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
  uint32_t probe;      // latency probe (kernel bench only): 2 = exit at entry, 1 = after the LDS
                       // table staging, 4 = after the tiles, 3 = after the done counter (no fold)
  CrcSeg seg[kMaxSeg];
};

struct CrcSegResult {
  uint32_t raw;
  uint32_t crc;
  uint32_t status;  // 0 not checked, 1 match, 2 mismatch; kCrcStatusPending until the kernel stores it
  uint32_t pad;
};
// A segment's status before its kernel stored the result: the kernels store
// raw / crc, fence at system scope, then status, so a host that sees a
// status other than this in host-mapped results also sees raw / crc -- and
// knows the slot's copy (ordered before the kernel on its stream) has landed
// (GpuSink: slot reuse without a HIP call on the receiving thread).
constexpr uint32_t kCrcStatusPending = 0xFFFFFFFFu;

struct CrcTables {
  uint32_t slice16[16][256];
  uint32_t lane_shift[7][4][256];  // [0..5]: shift by kCrcChunkBytes * 2^lv (wave tree); [6]: kCrcLaneGap
  uint32_t tile_shift[kCrcTileShiftLevels][4][256];  // shift by 4 KiB * 2^s
  // GF(2) shift matrices of the slot kernel (4 KiB tiles), column i = the
  // shift of the register value 1 << i: shift(s) = XOR_i bit_i(s) * col_i.
  //   lane_k[l]: lane l's 64-byte chunk ends 64 (63 - l) bytes before its
  //              tile's end;
  //   tile_k[d]: a tile ends 4 KiB * d bytes before its segment's last
  //              16-byte boundary (d < kCrcFusedMaxTiles).
  uint32_t lane_k[64][32];
  uint32_t tile_k[kCrcFusedMaxTiles][32];
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
// bound), 16 KiB above (bulk).  tile_log2 != 0 forces a size (tests, A/B).
void finalize_crc_batch(CrcBatch* b, uint32_t tile_log2 = 0);
// Words of tile scratch (header + tiles) a batch of up to `tiles` tiles needs.
inline uint64_t crc_scratch_words(uint64_t tiles) { return tiles + kCrcScratchHeader; }
// Host emulation of the kernels' math (same tables, same tile/lane/fold
// decomposition): the CPU test oracle.  fold_waves = 1 mirrors the fused
// epilogue, 8 the separate fold kernel.
// fold_waves = 0 mirrors the slot kernel (4 KiB tiles, <= kCrcFusedMaxTiles
// tiles): lane states through lane_k, tile values through tile_k, XOR.
CrcSegResult emulate_crc32c_segment(const uint8_t* addr, uint32_t len, const CrcTables& t, uint32_t expected,
                                    bool check, uint32_t tile_log2 = kCrcMaxTileLog2, int fold_waves = 8);
// s * (GF(2) matrix with columns col[0..31])
inline uint32_t crc_apply_columns(const uint32_t col[32], uint32_t s) {
  uint32_t r = 0;
  for (int i = 0; i < 32; ++i) r ^= col[i] & (0u - ((s >> i) & 1u));
  return r;
}

}  // namespace gcsb
