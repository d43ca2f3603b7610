// Plain-data types shared by the CRC32C kernels, their launchers and the
// host-side emulator (crc_emul.cc) that checks the kernel algorithm on CPU.
#pragma once
#include <cstdint>

namespace gcsb {

constexpr int kCrcTile = 4096;
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
  uint32_t lane_shift[7][4][256];  // shift by 16,32,64,128,256,512 and 1008 bytes
  uint32_t tile_shift[9][4][256];  // shift by 4096 * 2^s, s = 0..8 (last = 1 MiB)
};

// Number of full 16-byte pieces and 4 KiB tiles of a segment (host helper).
inline void crc_segment_geometry(uintptr_t addr, uint32_t len, uint32_t* ntiles) {
  if (len == 0) {
    *ntiles = 0;
    return;
  }
  uintptr_t a16 = addr & ~uintptr_t(15);
  uint64_t pieces = (addr + len - a16 + 15) / 16;
  uint64_t full = pieces - 1;
  *ntiles = static_cast<uint32_t>((full + 255) / 256);
}

// Host emulation of K1+K2 (same tables, same tile/lane decomposition) — the
// CPU test oracle for the kernel math.
void build_crc_tables(CrcTables* t);
// Fills seg.tile_base/ntiles/fixup and batch.total_tiles.
void finalize_crc_batch(CrcBatch* b);
CrcSegResult emulate_crc32c_segment(const uint8_t* addr, uint32_t len, const CrcTables& t, uint32_t expected,
                                    bool check);

}  // namespace gcsb
