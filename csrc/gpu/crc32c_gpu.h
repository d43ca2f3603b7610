// CDNA4 CRC32C engine: host-side types and launchers for the kernels in
// crc32c_kernels.hip.  [new] — the reference verifies CRC32C only inside the
// Go storage library on the host.
//
// A "segment" is one contiguous device byte range [addr, addr+len) whose
// CRC32C is wanted (one gRPC ChecksummedData message, or the part of it that
// landed in one ring slot, or one slot's share of an HTTP body).  A batch of up
// to kMaxSeg segments is ONE launch on the caller's stream when every segment
// fits kCrcFusedMaxTiles tiles (always true for ring slots):
//   crc32c_tiles_kernel : every wave CRCs one tile (4 or 16 KiB; 64 lanes x
//                         64-byte chunks, slice-by-16 + gap/tree shift tables
//                         staged in LDS, 6-level wave tree), tiles
//                         right-aligned to the segment end so a ragged head is
//                         just leading zeros (free for a raw CRC); the last
//                         workgroup to finish then folds each segment (one
//                         wave per segment: Horner + wave tree with LDS shift
//                         tables), adds the 1..16-byte tail in parallel,
//                         applies the init/xorout fixup and compares with the
//                         expected CRC, writing {raw, crc, status} to
//                         host-mapped memory.
// Longer segments add crc32c_fold_kernel (8 waves per segment) after the
// tiles.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gpu/crc_types.h"

namespace gcsb {

// Per-device, lazily uploaded tables.
const CrcTables* device_crc_tables(int device);

// Enqueue the batch (finalize_crc_batch first).  d_scratch: from
// crc_scratch_alloc(>= batch.total_tiles); batches sharing one scratch must be
// stream-ordered (its header word is the fused kernel's completion counter).
void launch_crc32c_batch(const CrcBatch& b, const CrcTables* d_tables, uint32_t* d_scratch,
                         CrcSegResult* d_results, hipStream_t stream);
uint32_t* crc_scratch_alloc(uint64_t tiles);

// Kernel variant selection for launch_crc32c_batch, process-wide.  The
// defaults are the measured winners; the others stay reachable for kernel
// A/Bs and their tests (scripts/crc_kernel_bench.py, tests/test_gpu_crc32c.py):
//   slot_waves    waves per slot-kernel workgroup (1, 2, 4, 8; 0 = by size)
//   xor_arrival   slot kernel: 64-bit XOR arrival words per counter group
//                 (false = per-tile stores + done counters for every batch)
// Measured and dropped (round 5, removed in round 6; git history and
// profiles/ keep them): an int8-MFMA tile kernel (2.9 TB/s against the table
// kernels' 3.9, profiles/r2_crc_mfma, r5_kernels), bank-replicated nibble
// tables (3.2 TB/s), the round-2 fused tile kernel for slot batches.
struct CrcLaunchOptions {
  int slot_waves = 0;
  bool xor_arrival = true;
  // slot kernel: stage slice-by-8 tables (8 KiB, T0..T7) instead of
  // slice-by-16 (16 KiB): the L2-cold stage in the read pipeline.  8.58-8.62
  // against 8.78-8.79 us per 1 MiB slot, min 6.5 against 7.0-7.3
  // (profiles/r4_crc8)
  bool slice8 = true;
  // bulk (non-fused) batches: bank-private slice-by-4 tables, conflict-free
  // lookups (crc32c_tiles_bp_kernel): 3.85-3.99 against 3.24-3.71 TB/s
  // (4 / 16 KiB tiles, profiles/r5_kernels)
  bool bank_private = true;
};
void set_crc_launch_options(const CrcLaunchOptions& o);
CrcLaunchOptions crc_launch_options();

// Pattern kernels (K3): object bytes of the synthetic content (csrc/core/content.h).
void launch_fill_pattern(uint8_t* dst, uint64_t n, uint64_t rot, uint64_t obj_off, hipStream_t stream);
// Counts mismatching bytes into *d_count (uint64) and records the first index.
void launch_verify_pattern(const uint8_t* src, uint64_t n, uint64_t rot, uint64_t obj_off,
                           unsigned long long* d_count, unsigned long long* d_first, hipStream_t stream);

void hip_check(hipError_t e, const char* what);

}  // namespace gcsb
