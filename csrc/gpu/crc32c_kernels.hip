// CDNA4 (gfx950) CRC32C kernels + synthetic-pattern fill/verify kernels.
// Geometry in crc_types.h.  Wave64 throughout: a wave owns a tile of R x 4 KiB
// (R = 1 or 4), read in R rounds where lane l takes its own contiguous 64-byte
// chunk (4 x global_load_dwordx4; each 128-byte line is consumed by two lanes
// within 4 consecutive loads, so L1 absorbs the 16 B-per-lane pattern).  The
// data has no reuse and never touches LDS; the LDS holds the 44 KiB of lookup
// tables: slice-by-16 (16 lookups per 16 B), one gap-shift table (a lane's
// state jumps 4032 B to its next chunk) and 6 wave-tree shift tables.
//
// One launch per ring slot (round 2): the tile kernel's last workgroup to
// finish (a "workgroups done" counter in the tile scratch, release/acquire
// fences at agent scope so tiles written on other XCDs' L2s are visible)
// restages the tile-fold shift tables into its LDS and folds every segment,
// one wave per segment: Horner over 64-tile strides, a 6-level wave tree, the
// 1..16-byte tail as one independent slice-by-r lookup per lane + an XOR
// reduction, the init/xorout fixup and the compare against the server's CRC,
// written to host-mapped memory.  Round 1 ran a second kernel for that fold
// with its shift tables read from global memory (7.1 us per slot, as long as
// the tile kernel; profiles/r1_bench_sliced4_kernel_stats.csv).  Segments over
// kCrcFusedMaxTiles tiles (bulk gpu_crc32c of large buffers) keep a separate
// fold kernel, 8 waves per segment, tables in LDS.
//
// Measured history (profiles/r1_k1, 1 GiB in 32 MiB segments): 4 KiB tiles
// with 16 B-strided lanes 2.4 TB/s -> lane-contiguous 256 B runs 3.0-3.1 TB/s
// -> 64 B chunks in 4 KiB rounds (16 KiB tiles) 3.5-3.7 TB/s.  Random
// ds_read_b32 table lookups cost ~4 bank-conflict cycles per instruction; a
// conflict-free variant (nibble tables replicated per bank) removed them but
// doubled the lookups and ran at 3.2 TB/s, so it was dropped in round 2.
// Round 5: byte tables replicated per bank (slice-by-4, 128 KiB, one lookup
// per byte, no conflicts) for bulk batches: 3.85-3.99 TB/s.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <string>

#include "core/content.h"
#include "core/crc32c.h"
#include "gpu/crc32c_gpu.h"

namespace gcsb {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

namespace {

constexpr int kThreads = 512;                      // 8 waves (tiles) per workgroup: amortise the table fill
constexpr int kWaves = kThreads / 64;
constexpr int kSliceWords = 16 * 256;
constexpr int kFoldLevels = 7;                     // fused fold: 1..64-tile shifts (levels 0..6)
constexpr int kK2Levels = 10;                      // 8-wave fold: levels 0..9 (512-tile Horner stride)

__device__ __forceinline__ uint32_t shift4(const uint32_t* __restrict__ tab, uint32_t s) {
  return tab[s & 0xff] ^ tab[256 + ((s >> 8) & 0xff)] ^ tab[512 + ((s >> 16) & 0xff)] ^ tab[768 + (s >> 24)];
}

// state advanced over 16 bytes of data (slice-by-16; T_k = byte followed by k zeros)
__device__ __forceinline__ uint32_t update16(const uint32_t* __restrict__ sl, uint32_t state, uint4 v) {
  const uint32_t x = state ^ v.x;
  uint32_t c = sl[15 * 256 + (x & 0xff)] ^ sl[14 * 256 + ((x >> 8) & 0xff)] ^ sl[13 * 256 + ((x >> 16) & 0xff)] ^
               sl[12 * 256 + (x >> 24)];
  c ^= sl[11 * 256 + (v.y & 0xff)] ^ sl[10 * 256 + ((v.y >> 8) & 0xff)] ^ sl[9 * 256 + ((v.y >> 16) & 0xff)] ^
       sl[8 * 256 + (v.y >> 24)];
  c ^= sl[7 * 256 + (v.z & 0xff)] ^ sl[6 * 256 + ((v.z >> 8) & 0xff)] ^ sl[5 * 256 + ((v.z >> 16) & 0xff)] ^
       sl[4 * 256 + (v.z >> 24)];
  c ^= sl[3 * 256 + (v.w & 0xff)] ^ sl[2 * 256 + ((v.w >> 8) & 0xff)] ^ sl[1 * 256 + ((v.w >> 16) & 0xff)] ^
       sl[0 * 256 + (v.w >> 24)];
  return c;
}

// The same 16 bytes as two slice-by-8 steps (tables T0..T7 only: half the
// LDS staging per workgroup, twice the dependent steps per lane).
__device__ __forceinline__ uint32_t update16_s8(const uint32_t* __restrict__ sl, uint32_t state, uint4 v) {
  const uint32_t x = state ^ v.x;
  uint32_t c = sl[7 * 256 + (x & 0xff)] ^ sl[6 * 256 + ((x >> 8) & 0xff)] ^ sl[5 * 256 + ((x >> 16) & 0xff)] ^
               sl[4 * 256 + (x >> 24)] ^ sl[3 * 256 + (v.y & 0xff)] ^ sl[2 * 256 + ((v.y >> 8) & 0xff)] ^
               sl[1 * 256 + ((v.y >> 16) & 0xff)] ^ sl[0 * 256 + (v.y >> 24)];
  const uint32_t z = c ^ v.z;
  c = sl[7 * 256 + (z & 0xff)] ^ sl[6 * 256 + ((z >> 8) & 0xff)] ^ sl[5 * 256 + ((z >> 16) & 0xff)] ^
      sl[4 * 256 + (z >> 24)] ^ sl[3 * 256 + (v.w & 0xff)] ^ sl[2 * 256 + ((v.w >> 8) & 0xff)] ^
      sl[1 * 256 + ((v.w >> 16) & 0xff)] ^ sl[0 * 256 + (v.w >> 24)];
  return c;
}

__device__ __forceinline__ uint32_t mask_low_bytes(uint32_t w, int keep_from) {
  // zero bytes [0, keep_from) of a little-endian word (keep_from in 0..4)
  if (keep_from <= 0) return w;
  if (keep_from >= 4) return 0;
  return w & (0xFFFFFFFFu << (8 * keep_from));
}

__device__ __forceinline__ void stage(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, int words) {
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  for (int i = threadIdx.x; i < words / 4; i += blockDim.x) d4[i] = s4[i];
}

// The tile's 16-byte pieces for this lane (R rounds x kCrcChunkPieces).
template <int R>
__device__ __forceinline__ void load_tile(const CrcBatch& b, uint32_t s, uint32_t gt, int lane,
                                          uint4 (&v)[R * kCrcChunkPieces]) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(b.seg[s].addr);
  const uint32_t len = b.seg[s].len;
  const uint32_t t = gt - b.seg[s].tile_base;
  const uintptr_t a16 = addr & ~uintptr_t(15);
  const uint64_t full = (addr + len - a16 + 15) / 16 - 1;
  const intptr_t vend = static_cast<intptr_t>(a16 + 16 * full);
  const intptr_t tstart = vend - (static_cast<intptr_t>(R) * kCrcRoundBytes) * static_cast<intptr_t>(b.seg[s].ntiles - t);
#pragma unroll
  for (int k = 0; k < R; ++k)
#pragma unroll
    for (int j = 0; j < kCrcChunkPieces; ++j) {
      const intptr_t p = tstart + kCrcRoundBytes * k + kCrcChunkBytes * lane + 16 * j;
      uint4 x = make_uint4(0, 0, 0, 0);
      if (p + 16 > static_cast<intptr_t>(addr)) x = *reinterpret_cast<const uint4*>(p);
      if (p < static_cast<intptr_t>(addr) && p + 16 > static_cast<intptr_t>(addr)) {
        const int h = static_cast<int>(static_cast<intptr_t>(addr) - p);  // 1..15 leading bytes to zero
        x.x = mask_low_bytes(x.x, h);
        x.y = mask_low_bytes(x.y, h - 4);
        x.z = mask_low_bytes(x.z, h - 8);
        x.w = mask_low_bytes(x.w, h - 12);
      }
      v[k * kCrcChunkPieces + j] = x;
    }
}

// The lane's CRC register over its chunks of the tile.
template <int R, bool kS8 = false>
__device__ __forceinline__ uint32_t lane_chain(const uint4 (&v)[R * kCrcChunkPieces], const uint32_t* sl,
                                               const uint32_t* lane_shift, int lane) {
  uint32_t state = 0;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    if (k) state = shift4(lane_shift + 6 * 1024, state);  // over the 4032-byte gap to this lane's next chunk
#pragma unroll
    for (int j = 0; j < kCrcChunkPieces; ++j) {
      if constexpr (kS8)
        state = update16_s8(sl, state, v[k * kCrcChunkPieces + j]);
      else
        state = update16(sl, state, v[k * kCrcChunkPieces + j]);
    }
  }
  return state;
}

// Tile `gt` of the batch: per-lane register.  Pieces before the segment
// start read as zeros (free for a raw CRC); the piece straddling it is masked.
// Tiles are right-aligned to the segment end, so only the first tile of a
// segment has such a head.
template <int R>
__device__ __forceinline__ uint32_t lane_state(const CrcBatch& b, uint32_t s, uint32_t gt, const uint32_t* sl,
                                               const uint32_t* lane_shift, int lane) {
  uint4 v[R * kCrcChunkPieces];
  load_tile<R>(b, s, gt, lane, v);
  // keep all the tile's loads in flight before the first lookup (the
  // scheduler otherwise sinks them into the lookup chain)
  __builtin_amdgcn_sched_barrier(0);
  return lane_chain<R>(v, sl, lane_shift, lane);
}

// wave tree: lane l's last chunk ends 64 (63 - l) bytes before the tile end
__device__ __forceinline__ uint32_t wave_tree(uint32_t state, const uint32_t* lane_shift, int lane) {
#pragma unroll
  for (int lv = 0; lv < 6; ++lv) {
    const uint32_t other = __shfl_down(state, 1 << lv, 64);
    const uint32_t shifted = shift4(lane_shift + lv * 1024, state);
    if ((lane & ((2 << lv) - 1)) == 0) state = shifted ^ other;
  }
  return state;
}

template <int R>
__device__ __forceinline__ uint32_t tile_crc(const CrcBatch& b, uint32_t s, uint32_t gt, const uint32_t* sl,
                                             const uint32_t* lane_shift, int lane) {
  return wave_tree(lane_state<R>(b, s, gt, sl, lane_shift, lane), lane_shift, lane);
}

// The last 1..16 bytes of a segment (after its tiles) folded into `raw`: lane
// i < r looks up slice16[r-1-i][byte_i ^ state byte i] independently, an XOR
// reduction over 16 lanes combines them (slice-by-r).  Result in every lane.
__device__ __forceinline__ uint32_t add_tail(const CrcSeg& sg, uint32_t raw, const uint32_t* sl, int lane) {
  if (sg.len == 0) return raw;
  const uintptr_t addr = reinterpret_cast<uintptr_t>(sg.addr);
  const uintptr_t a16 = addr & ~uintptr_t(15);
  const uintptr_t e = addr + sg.len;
  const uintptr_t vend = a16 + 16 * ((e - a16 + 15) / 16 - 1);
  const uintptr_t p0 = vend > addr ? vend : addr;
  const int r = static_cast<int>(e - p0);
  uint32_t x = 0;
  if (lane < r) {
    const uint32_t sb = lane < 4 ? (raw >> (8 * lane)) & 0xff : 0u;
    x = sl[(r - 1 - lane) * 256 + ((*reinterpret_cast<const uint8_t*>(p0 + lane) ^ sb) & 0xff)];
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
  return x ^ (r < 4 ? raw >> (8 * r) : 0u);
}

// Split add_tail for prefetching: the segment's last r (1..16) bytes, byte
// `lane` of them in lanes < r (0 elsewhere)...
__device__ __forceinline__ uint32_t tail_byte(const CrcSeg& sg, int lane, int* r_out) {
  *r_out = 0;
  if (sg.len == 0) return 0u;
  const uintptr_t addr = reinterpret_cast<uintptr_t>(sg.addr);
  const uintptr_t a16 = addr & ~uintptr_t(15);
  const uintptr_t e = addr + sg.len;
  const uintptr_t vend = a16 + 16 * ((e - a16 + 15) / 16 - 1);
  const uintptr_t p0 = vend > addr ? vend : addr;
  const int r = static_cast<int>(e - p0);
  *r_out = r;
  return lane < r ? static_cast<uint32_t>(*reinterpret_cast<const uint8_t*>(p0 + lane)) : 0u;
}

// ... folded into `raw` (slice-by-r, one independent lookup per lane)
__device__ __forceinline__ uint32_t fold_tail(uint32_t byte, int r, uint32_t raw, const uint32_t* tab, int lane) {
  if (r == 0) return raw;
  uint32_t x = 0;
  if (lane < r) {
    const uint32_t sb = lane < 4 ? (raw >> (8 * lane)) & 0xff : 0u;
    const uint32_t bv = (byte ^ sb) & 0xff;
    const int m = r - 1 - lane;  // slice16 table index
    x = tab[m * 256 + bv];
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
  return x ^ (r < 4 ? raw >> (8 * r) : 0u);
}

// Result store for (host-mapped) result slots: raw / crc first, then, after
// a system-scope fence, the status word the host polls (kCrcStatusPending).
__device__ __forceinline__ void store_result(CrcSegResult* o, const CrcSegResult& r) {
  o->raw = r.raw;
  o->crc = r.crc;
  o->pad = 0;
  __threadfence_system();
  __hip_atomic_store(&o->status, r.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ CrcSegResult seg_result(const CrcSeg& sg, uint32_t raw) {
  const uint32_t crc = raw ^ sg.fixup;
  CrcSegResult r;
  r.raw = raw;
  r.crc = crc;
  r.status = (sg.flags & 1) ? (crc == sg.expected ? 1u : 2u) : 0u;
  r.pad = 0;
  return r;
}

// One wave folds one segment's tiles (ntiles <= kCrcFusedMaxTiles): lane k
// takes tiles T-1-(k + 64 m) by Horner (64-tile shift), then the wave tree.
// ts = tile_shift tables, level 0 = a shift by one tile.  Tile values are
// loaded 8 at a time ahead of their Horner steps (one memory latency per 8
// steps instead of one per step).  kCoherent: tiles written by other
// workgroups in this launch -> agent-scope loads (sc1: past this XCD's L2).
template <bool kCoherent>
__device__ __forceinline__ uint32_t fold_wave(const CrcSeg& sg, const uint32_t* __restrict__ tiles,
                                              const uint32_t* ts, int lane) {
  const uint32_t T = sg.ntiles;
  const uint32_t* tp = tiles + sg.tile_base;
  uint32_t acc = 0;
  const int M = static_cast<int>((T + 63) >> 6);
  for (int m0 = M - 1; m0 >= 0; m0 -= 8) {
    uint32_t tv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 - i;
      const uint32_t j = static_cast<uint32_t>(lane) + 64u * static_cast<uint32_t>(m);
      tv[i] = 0;
      if (m >= 0 && j < T) {
        if constexpr (kCoherent)
          tv[i] = __hip_atomic_load(tp + (T - 1 - j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
          tv[i] = tp[T - 1 - j];
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (m0 - i >= 0) acc = shift4(ts + 6 * 1024, acc) ^ tv[i];
  }
#pragma unroll
  for (int lv = 0; lv < 6; ++lv) {
    const uint32_t other = __shfl_down(acc, 1 << lv, 64);
    if ((lane & ((2 << lv) - 1)) == 0) acc ^= shift4(ts + lv * 1024, other);
  }
  return __shfl(acc, 0, 64);
}

// Tile kernel; kFused: the last workgroup to finish folds every segment.
template <int R, bool kFused>
__global__ __launch_bounds__(kThreads) void crc32c_tiles_kernel(const CrcBatch b, const CrcTables* __restrict__ tabs,
                                                                uint32_t* __restrict__ scratch,
                                                                CrcSegResult* __restrict__ out) {
  // LDS: slice16 | 6 wave-tree shifts | gap shift (R > 1) | tile-fold shifts
  // (fused: staged up front with the rest, so the last workgroup folds at
  // once instead of restaging; 68 KiB for R = 1, 2 workgroups per CU)
  constexpr int kGapWords = R > 1 ? 1024 : 0;
  constexpr int kFoldWords = kFused ? kFoldLevels * 1024 : 0;
  constexpr int kTreeWords = 6 * 1024;
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kSliceWords + kTreeWords + kGapWords + kFoldWords];
  __shared__ uint32_t s_last;
  if (b.probe == 2) return;
  stage(s_tab, &tabs->slice16[0][0], kSliceWords);
  stage(s_tab + kSliceWords, &tabs->lane_shift[0][0][0], kTreeWords + kGapWords);
  if constexpr (kFused)
    stage(s_tab + kSliceWords + kTreeWords + kGapWords,
          &tabs->tile_shift[static_cast<int>(b.tile_log2) - kCrcMinTileLog2][0][0], kFoldWords);
  __syncthreads();
  if (b.probe == 1) return;
  const uint32_t* sl = s_tab;
  const uint32_t* lane_shift = s_tab + kSliceWords;
  uint32_t* tiles = scratch + kCrcScratchHeader;
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  // gt only grows, so the segment search resumes where the last tile left it
  uint32_t s = 0;
  for (uint32_t gt = blockIdx.x * kWaves + wave; gt < b.total_tiles; gt += nwaves) {
    while (s + 1 < b.nseg && b.seg[s + 1].tile_base <= gt) ++s;
    const uint32_t c = tile_crc<R>(b, s, gt, sl, lane_shift, lane);
    if (lane == 0) {
      if constexpr (kFused)  // written through to the agent coherence point (sc1): no L2 writeback needed
        __hip_atomic_store(tiles + gt, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        tiles[gt] = c;
    }
  }
  if (b.probe == 4) return;
  if constexpr (kFused) {
    // Every wave's tile stores must have completed (vmcnt 0) before thread 0
    // counts this workgroup done; __syncthreads alone does not wait for them.
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0)
      s_last = __hip_atomic_fetch_add(scratch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1
                   ? 1u : 0u;
    __syncthreads();
    if (!s_last) return;
    if (b.probe == 3) {
      if (threadIdx.x == 0) __hip_atomic_store(scratch, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    for (uint32_t g = wave; g < b.nseg; g += kWaves) {
      const CrcSeg& sg = b.seg[g];
      uint32_t raw = fold_wave<true>(sg, tiles, s_tab + kSliceWords + kTreeWords + kGapWords, lane);
      raw = add_tail(sg, raw, sl, lane);
      if (lane == 0) store_result(out + g, seg_result(sg, raw));
    }
    if (threadIdx.x == 0) __hip_atomic_store(scratch, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Bank-private slice-by-4 (bulk, non-fused, the default): each 32-lane half
// of a wave reads its lookups from 32 private copies of T0..T3, lane l only
// from bank l, so ds_read_b32 never conflicts.  The slice-by-16 tables above
// cost ~4 extra LDS cycles per lookup and left the waves 42% of their cycles
// waiting on LDS (SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES); here 2%
// (profiles/r5_kernels).  One lookup per byte as before; 128 KiB of tables +
// the shift tables, so one 16-wave workgroup per CU stages them once and
// grid-strides over the tiles.  A 16-copy variant (2-way conflicts, shift
// tables from global memory, two workgroups per CU) measured slower.
constexpr int kBpThreads = 1024;
constexpr int kBpWaves = kBpThreads / 64;

template <int kRep>
__device__ __forceinline__ uint32_t step4_bp(const uint32_t* __restrict__ bp, uint32_t x) {
  return bp[(3 * 256 + (x & 0xff)) * kRep] ^ bp[(2 * 256 + ((x >> 8) & 0xff)) * kRep] ^
         bp[(1 * 256 + ((x >> 16) & 0xff)) * kRep] ^ bp[(x >> 24) * kRep];
}

template <int R, int kRep>
__global__ __launch_bounds__(kBpThreads) void crc32c_tiles_bp_kernel(const CrcBatch b, const CrcTables* __restrict__ tabs,
                                                                   uint32_t* __restrict__ scratch) {
  constexpr int kBpWords = 4 * 256 * kRep;
  static_assert(kRep == 32, "one table copy per ds_read_b32 bank");
  constexpr int kShWords = 6 * 1024 + (R > 1 ? 1024 : 0);
  __shared__ __attribute__((aligned(16))) uint32_t s_bp[kBpWords];
  __shared__ __attribute__((aligned(16))) uint32_t s_sh[kShWords];
  // latency probes of the kernel bench (CrcBatch::probe), as the other tile
  // kernels: 2 = exit at entry, 1 = after the table staging; 4 (after the
  // tiles) is where this kernel ends anyway
  const uint32_t probe = b.probe & 0xffu;
  if (probe == 2) return;
  // word i = T_(i / (256 kRep))[(i / kRep) & 255], bank i % kRep
  for (int i = threadIdx.x; i < kBpWords; i += blockDim.x) s_bp[i] = tabs->slice16[i / (256 * kRep)][(i / kRep) & 255];
  stage(s_sh, &tabs->lane_shift[0][0][0], kShWords);
  __syncthreads();
  if (probe == 1) return;
  const uint32_t* sh = s_sh;
  const int lane = threadIdx.x & 63;
  const uint32_t* bp = s_bp + (lane & (kRep - 1));
  uint32_t* tiles = scratch + kCrcScratchHeader;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kBpWaves;
  uint32_t s = 0;
  for (uint32_t gt = blockIdx.x * kBpWaves + wave; gt < b.total_tiles; gt += nwaves) {
    while (s + 1 < b.nseg && b.seg[s + 1].tile_base <= gt) ++s;
    uint4 v[R * kCrcChunkPieces];
    load_tile<R>(b, s, gt, lane, v);
    __builtin_amdgcn_sched_barrier(0);
    // the R chunks as R independent chains, interleaved (a slice-by-4 chain
    // is 16 dependent lookups per 64-byte chunk), then combined: a chunk's
    // register moves 4096 B (the 4032-byte gap + the next 64-byte chunk)
    // before the next chunk's is XORed in
    uint32_t st[R];
#pragma unroll
    for (int k = 0; k < R; ++k) st[k] = 0;
#pragma unroll
    for (int j = 0; j < kCrcChunkPieces; ++j) {
#pragma unroll
      for (int k = 0; k < R; ++k) st[k] = step4_bp<kRep>(bp, st[k] ^ v[k * kCrcChunkPieces + j].x);
#pragma unroll
      for (int k = 0; k < R; ++k) st[k] = step4_bp<kRep>(bp, st[k] ^ v[k * kCrcChunkPieces + j].y);
#pragma unroll
      for (int k = 0; k < R; ++k) st[k] = step4_bp<kRep>(bp, st[k] ^ v[k * kCrcChunkPieces + j].z);
#pragma unroll
      for (int k = 0; k < R; ++k) st[k] = step4_bp<kRep>(bp, st[k] ^ v[k * kCrcChunkPieces + j].w);
    }
    uint32_t state = st[0];
#pragma unroll
    for (int k = 1; k < R; ++k) state = shift4(sh, shift4(sh + 6 * 1024, state)) ^ st[k];
    const uint32_t c = wave_tree(state, sh, lane);
    if (lane == 0) tiles[gt] = c;
  }
}

__device__ __forceinline__ uint32_t xor_over_lanes(uint32_t x, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
  return x;
}

// Slot kernel (4 KiB tiles, segments <= kCrcFusedMaxTiles tiles: every ring
// slot).  Same lane chains as tile_crc<1>, but no lookup-table wave tree and
// no Horner fold: CRC shifts are GF(2)-linear, so each lane's state goes
// straight to its tile's end through a 32x32 bit matrix held in 32 VGPRs
// (lane_k, loaded once per wave), the XOR over the 64 lanes is the tile's raw
// CRC, and one more matrix (tile_k[d], a coalesced 128 B load issued with the
// tile's data) moves it to the segment end.  Each wave stores that
// contribution (write-through to the device coherence point); the last
// workgroup, found through a two-level done counter, XORs each segment's
// contributions (independent loads, no chain), adds the 1..16-byte tail,
// fixes up, compares and writes the result.
// Decomposition of the round-2 fused tile kernel on a 2 MiB slot
// (profiles/r2_crc_slot): 2.7 us in tiles (64 CUs busy, 88 LDS lookups per
// lane, a 6-level lookup chain), 1.0 us on the done counter, 2.5 us in the
// last workgroup's Horner + tree fold.  W (waves per workgroup) is picked so
// the grid puts a tile on every CU.
template <int W, bool kS8 = false>
__global__ __launch_bounds__(64 * W) void crc32c_slot_kernel(const CrcBatch b, const CrcTables* __restrict__ tabs,
                                                            uint32_t* __restrict__ scratch,
                                                            CrcSegResult* __restrict__ out) {
  constexpr int kTabWords = kS8 ? 8 * 256 : kSliceWords;
  // the tail fold looks up T0..T15: from L2 when only T0..T7 were staged
  const uint32_t* tail_tab = kS8 ? &tabs->slice16[0][0] : nullptr;
  __shared__ __attribute__((aligned(16))) uint32_t s_sl[kTabWords];
  __shared__ uint32_t s_last;
  const uint32_t probe = b.probe & 0xffu;  // bit 8: A/B switch, per-tile stores + counters only
  if (probe == 2) return;
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the first tile's data and matrix go out before the tables: their memory
  // latency overlaps the staging's instead of following it (the slot's bytes
  // were just written by SDMA, the tables are L2-cold between slots)
  const uint32_t gt0 = blockIdx.x * W + wave;
  uint32_t s = 0;
  uint4 v[kCrcChunkPieces];
  uint32_t kt = 0;
  if (gt0 < b.total_tiles) {
    while (s + 1 < b.nseg && b.seg[s + 1].tile_base <= gt0) ++s;
    kt = tabs->tile_k[b.seg[s].ntiles - 1 - (gt0 - b.seg[s].tile_base)][lane & 31];
    load_tile<1>(b, s, gt0, lane, v);
  }
  // this lane's chunk -> tile end: 32 matrix columns, in registers
  uint32_t kl[32];
  {
    const uint4* kp = reinterpret_cast<const uint4*>(&tabs->lane_k[lane][0]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint4 q = kp[j];
      kl[4 * j] = q.x;
      kl[4 * j + 1] = q.y;
      kl[4 * j + 2] = q.z;
      kl[4 * j + 3] = q.w;
    }
  }
  stage(s_sl, &tabs->slice16[0][0], kTabWords);
  __syncthreads();
  if (probe == 1) return;
  uint32_t* tiles = scratch + kCrcScratchHeader;
  // One segment (every slot that does not straddle two objects) and at most
  // 32 workgroups per counter group: no per-tile stores.  Each workgroup's
  // contribution and its arrival bit go into one 64-bit atomic XOR per level
  // (low word: XOR of contributions, high word: arrival mask); the returned
  // old value tells the last arriver the whole XOR.  Two device-scope round
  // trips instead of store + wait + counter + counter + loads.
  const uint32_t groups = gridDim.x < kCrcCounterGroups ? gridDim.x : kCrcCounterGroups;
  const bool xor_path = b.nseg == 1 && gridDim.x <= 32u * groups && !(b.probe & 0x100u);
  int tail_r = 0;
  const uint32_t tail_b = xor_path && wave == 0 ? tail_byte(b.seg[0], lane, &tail_r) : 0u;
  uint32_t wsum = 0;
  for (uint32_t gt = gt0; gt < b.total_tiles; gt += gridDim.x * W) {
    if (gt != gt0) {
      while (s + 1 < b.nseg && b.seg[s + 1].tile_base <= gt) ++s;
      kt = tabs->tile_k[b.seg[s].ntiles - 1 - (gt - b.seg[s].tile_base)][lane & 31];
      load_tile<1>(b, s, gt, lane, v);
      __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t state = lane_chain<1, kS8>(v, s_sl, nullptr, lane);
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) c ^= kl[i] & (0u - ((state >> i) & 1u));
    c = xor_over_lanes(c, 64);  // the tile's raw CRC, in every lane
    uint32_t x = lane < 32 ? (kt & (0u - ((c >> lane) & 1u))) : 0u;
    x = xor_over_lanes(x, 32);
    if (xor_path)
      wsum ^= x;
    else if (lane == 0)
      __hip_atomic_store(tiles + gt, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (probe == 4) return;
  if (xor_path) {
    __shared__ uint32_t s_part[W];
    __shared__ uint32_t s_raw;
    if (lane == 0) s_part[wave] = wsum;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t mine = 0;
#pragma unroll
      for (int i = 0; i < W; ++i) mine ^= s_part[i];
      const uint32_t j = blockIdx.x % groups;
      const uint32_t m = blockIdx.x / groups;
      const uint32_t members = gridDim.x / groups + (j < gridDim.x % groups ? 1u : 0u);
      const uint32_t full = members >= 32 ? ~0u : (1u << members) - 1u;
      // 8-byte aligned words inside the header's group / root slots
      auto word = [](uint32_t* p) {
        return reinterpret_cast<uint64_t*>((reinterpret_cast<uintptr_t>(p) + 8 + 7) & ~uintptr_t(7));
      };
      uint64_t* gw = word(scratch + kCrcCounterStride * (1 + j));
      uint32_t last = 0;
      const uint64_t og = __hip_atomic_fetch_xor(gw, (uint64_t{1} << (32 + m)) | mine, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
      if ((static_cast<uint32_t>(og >> 32) ^ (1u << m)) == full) {
        __hip_atomic_store(gw, uint64_t{0}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t gx = static_cast<uint32_t>(og) ^ mine;
        const uint32_t gfull = groups >= 32 ? ~0u : (1u << groups) - 1u;
        uint64_t* rw = word(scratch);
        const uint64_t orr = __hip_atomic_fetch_xor(rw, (uint64_t{1} << (32 + j)) | gx, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if ((static_cast<uint32_t>(orr >> 32) ^ (1u << j)) == gfull) {
          __hip_atomic_store(rw, uint64_t{0}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_raw = static_cast<uint32_t>(orr) ^ gx;
          last = 1;
        }
      }
      s_last = last;
    }
    __syncthreads();
    if (!s_last || probe == 3 || wave != 0) return;
    const uint32_t raw = fold_tail(tail_b, tail_r, s_raw, kS8 ? tail_tab : s_sl, lane);
    if (lane == 0) store_result(out + 0, seg_result(b.seg[0], raw));
    return;
  }
  // this workgroup's stores complete before it counts itself done
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    // two-level done counter: a group counter per 1/16 of the grid, the
    // group's last workgroup counts the group on the root counter
    const uint32_t groups = gridDim.x < kCrcCounterGroups ? gridDim.x : kCrcCounterGroups;
    const uint32_t j = blockIdx.x % groups;
    const uint32_t members = gridDim.x / groups + (j < gridDim.x % groups ? 1u : 0u);
    uint32_t* gc = scratch + kCrcCounterStride * (1 + j);
    uint32_t last = 0;
    if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == members - 1) {
      __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(scratch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1) {
        __hip_atomic_store(scratch, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = 1;
      }
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last || probe == 3) return;
  for (uint32_t g = wave; g < b.nseg; g += W) {
    const CrcSeg& sg = b.seg[g];
    const uint32_t* tp = tiles + sg.tile_base;
    // the tail bytes and every contribution in flight at once (<= 16 per
    // lane), then the XORs: a rolled loop waits one device-scope round trip
    // per step (3.1 us for 8 steps)
    int r = 0;
    const uint32_t tb = tail_byte(sg, lane, &r);
    uint32_t v[kCrcFusedMaxTiles / 64];
#pragma unroll
    for (int k = 0; k < static_cast<int>(kCrcFusedMaxTiles / 64); ++k) {
      const uint32_t j = static_cast<uint32_t>(lane) + 64u * static_cast<uint32_t>(k);
      v[k] = j < sg.ntiles ? __hip_atomic_load(tp + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < static_cast<int>(kCrcFusedMaxTiles / 64); ++k) acc ^= v[k];
    uint32_t raw = xor_over_lanes(acc, 64);
    raw = fold_tail(tb, r, raw, kS8 ? tail_tab : s_sl, lane);
    if (lane == 0) store_result(out + g, seg_result(sg, raw));
  }
}

// Separate fold for long segments: one 8-wave workgroup per segment, Horner
// over 512-tile strides, wave tree, then a 3-level tree across the waves.
__global__ __launch_bounds__(kThreads) void crc32c_fold_kernel(const CrcBatch b, const CrcTables* __restrict__ tabs,
                                                               const uint32_t* __restrict__ scratch,
                                                               CrcSegResult* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kSliceWords + kK2Levels * 1024];
  __shared__ uint32_t part[kWaves];
  const uint32_t g = blockIdx.x;
  if (g >= b.nseg) return;
  const int lvl0 = static_cast<int>(b.tile_log2) - kCrcMinTileLog2;
  stage(s_tab, &tabs->slice16[0][0], kSliceWords);
  stage(s_tab + kSliceWords, &tabs->tile_shift[lvl0][0][0], kK2Levels * 1024);
  __syncthreads();
  const uint32_t* ts = s_tab + kSliceWords;
  const CrcSeg& sg = b.seg[g];
  const uint32_t T = sg.ntiles;
  const uint32_t* tp = scratch + kCrcScratchHeader + sg.tile_base;
  const int k = threadIdx.x;
  const int lane = k & 63;
  uint32_t acc = 0;
  const int M = static_cast<int>((T + kThreads - 1) / kThreads);
  for (int m = M - 1; m >= 0; --m) {
    acc = shift4(ts + 9 * 1024, acc);
    const uint32_t j = static_cast<uint32_t>(k) + static_cast<uint32_t>(kThreads) * static_cast<uint32_t>(m);
    if (j < T) acc ^= tp[T - 1 - j];
  }
#pragma unroll
  for (int lv = 0; lv < 6; ++lv) {
    const uint32_t other = __shfl_down(acc, 1 << lv, 64);
    if ((lane & ((2 << lv) - 1)) == 0) acc ^= shift4(ts + lv * 1024, other);
  }
  if (lane == 0) part[k >> 6] = acc;
  __syncthreads();
  if (k < 64) {
    uint32_t p = lane < kWaves ? part[lane] : 0u;
#pragma unroll
    for (int lv = 0; lv < 3; ++lv) {
      const uint32_t other = __shfl_down(p, 1 << lv, 64);
      if ((lane & ((2 << lv) - 1)) == 0) p ^= shift4(ts + (6 + lv) * 1024, other);
    }
    uint32_t raw = __shfl(p, 0, 64);
    raw = add_tail(sg, raw, s_tab, lane);
    if (lane == 0) store_result(out + g, seg_result(sg, raw));
  }
}

__device__ __forceinline__ uint8_t obj_byte(uint64_t q) {
  return pattern_byte(kPatternSeed, q);
}

__global__ __launch_bounds__(256) void fill_pattern_kernel(uint8_t* __restrict__ dst, uint64_t n, uint64_t rot,
                                                           uint64_t obj_off) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g * 16 < n; g += stride) {
    const uint64_t b0 = g * 16;
    uint64_t q = (obj_off + b0 + rot) % kPatternLen;
    uint8_t v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      v[e] = obj_byte(q);
      q = (q + 1 == kPatternLen) ? 0 : q + 1;
    }
    if (b0 + 16 <= n && (reinterpret_cast<uintptr_t>(dst + b0) & 15) == 0) {
      uint4 w;
      __builtin_memcpy(&w, v, 16);
      *reinterpret_cast<uint4*>(dst + b0) = w;
    } else {
      for (int e = 0; e < 16 && b0 + e < n; ++e) dst[b0 + e] = v[e];
    }
  }
}

__global__ __launch_bounds__(256) void verify_pattern_kernel(const uint8_t* __restrict__ src, uint64_t n, uint64_t rot,
                                                             uint64_t obj_off, unsigned long long* count,
                                                             unsigned long long* first) {
  // same generation path as fill_pattern_kernel; per-block reduction, one
  // atomic pair per block
  __shared__ unsigned long long s_bad[256];
  __shared__ unsigned long long s_first[256];
  unsigned long long bad = 0, first_bad = ~0ull;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g * 16 < n; g += stride) {
    const uint64_t b0 = g * 16;
    uint64_t q = (obj_off + b0 + rot) % kPatternLen;
    uint8_t v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      v[e] = obj_byte(q);
      q = (q + 1 == kPatternLen) ? 0 : q + 1;
    }
    const int lim = (b0 + 16 <= n) ? 16 : static_cast<int>(n - b0);
    for (int e = 0; e < lim; ++e) {
      if (src[b0 + e] != v[e]) {
        ++bad;
        if (b0 + e < first_bad) first_bad = b0 + e;
      }
    }
  }
  s_bad[threadIdx.x] = bad;
  s_first[threadIdx.x] = first_bad;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) {
      s_bad[threadIdx.x] += s_bad[threadIdx.x + w];
      if (s_first[threadIdx.x + w] < s_first[threadIdx.x]) s_first[threadIdx.x] = s_first[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && s_bad[0]) {
    atomicAdd(count, s_bad[0]);
    atomicMin(first, s_first[0]);
  }
}

}  // namespace

const CrcTables* device_crc_tables(int device) {
  static std::mutex mu;
  static CrcTables* per_dev[64] = {nullptr};
  static CrcTables* host = nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (device < 0 || device >= 64) throw std::runtime_error("bad device index");
  if (!per_dev[device]) {
    if (!host) {
      host = new CrcTables();
      build_crc_tables(host);
    }
    int prev = 0;
    hip_check(hipGetDevice(&prev), "hipGetDevice");
    hip_check(hipSetDevice(device), "hipSetDevice");
    CrcTables* d = nullptr;
    hip_check(hipMalloc(reinterpret_cast<void**>(&d), sizeof(CrcTables)), "hipMalloc(tables)");
    hip_check(hipMemcpy(d, host, sizeof(CrcTables), hipMemcpyHostToDevice), "hipMemcpy(tables)");
    per_dev[device] = d;
    hip_check(hipSetDevice(prev), "hipSetDevice");
  }
  return per_dev[device];
}

void launch_crc32c_batch(const CrcBatch& b, const CrcTables* d_tables, uint32_t* d_scratch,
                         CrcSegResult* d_results, hipStream_t stream) {
  if (b.nseg == 0) return;
  uint32_t blocks = (b.total_tiles + kWaves - 1) / kWaves;
  if (blocks > 1024) blocks = 1024;  // grid-stride over the rest
  if (blocks == 0) blocks = 1;       // tail-only segments: the fused fold still runs
  const bool fused = b.max_seg_tiles <= kCrcFusedMaxTiles;
  const bool small = b.tile_log2 == static_cast<uint32_t>(kCrcMinTileLog2);
  const CrcLaunchOptions o = crc_launch_options();
  if (fused && small) {
    // waves per workgroup: enough workgroups to put a tile on every CU first,
    // but two waves from 1 MiB up (each workgroup stages the 16 KiB tables,
    // L2-cold between slots: 1 MiB slots in the read pipeline averaged 9.23 /
    // 8.62 / 8.79 / 10.74 us with 1 / 2 / 4 / 8 waves, profiles/r4_crcw)
    const uint32_t t = b.total_tiles;
    int w = t < 256 ? 1 : t <= 512 ? 2 : t <= 1024 ? 4 : 8;
    if (o.slot_waves == 1 || o.slot_waves == 2 || o.slot_waves == 4 || o.slot_waves == 8) w = o.slot_waves;
    uint32_t g = (t + w - 1) / w;
    if (g > 2048) g = 2048;
    const bool no_xor = !o.xor_arrival;
    CrcBatch bx;
    if (no_xor) {
      bx = b;
      bx.probe |= 0x100u;
    }
    if (g == 0) g = 1;
#define GCSB_SLOT(WV, S8) \
  hipLaunchKernelGGL((crc32c_slot_kernel<WV, S8>), dim3(g), dim3(64 * WV), 0, stream, no_xor ? bx : b, d_tables, \
                     d_scratch, d_results)
    if (o.slice8) {
      switch (w) {
        case 1: GCSB_SLOT(1, true); break;
        case 2: GCSB_SLOT(2, true); break;
        case 4: GCSB_SLOT(4, true); break;
        default: GCSB_SLOT(8, true); break;
      }
    } else {
      switch (w) {
        case 1: GCSB_SLOT(1, false); break;
        case 2: GCSB_SLOT(2, false); break;
        case 4: GCSB_SLOT(4, false); break;
        default: GCSB_SLOT(8, false); break;
      }
    }
#undef GCSB_SLOT
    hip_check(hipGetLastError(), "crc32c_slot_kernel");
    return;
  }
  if (fused) {  // 16 KiB tiles (batches over 4 MiB whose segments fold in one pass)
    hipLaunchKernelGGL((crc32c_tiles_kernel<4, true>), dim3(blocks), dim3(kThreads), 0, stream, b, d_tables,
                       d_scratch, d_results);
    hip_check(hipGetLastError(), "crc32c_tiles_kernel(fused)");
    return;
  }
  if (o.bank_private) {
    // a persistent grid: one workgroup per CU (128 KiB of tables each)
    static std::atomic<int> cu_count[64];  // per device, 0 = not asked yet
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
      cus = cu_count[dev].load(std::memory_order_relaxed);
      if (cus <= 0) {
        cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        cu_count[dev].store(cus, std::memory_order_relaxed);
      }
    }
    const uint32_t need = (b.total_tiles + kBpWaves - 1) / kBpWaves;
    const uint32_t g = std::max<uint32_t>(1, std::min<uint32_t>(need, static_cast<uint32_t>(std::max(cus, 1))));
    if (small)
      hipLaunchKernelGGL((crc32c_tiles_bp_kernel<1, 32>), dim3(g), dim3(kBpThreads), 0, stream, b, d_tables, d_scratch);
    else
      hipLaunchKernelGGL((crc32c_tiles_bp_kernel<4, 32>), dim3(g), dim3(kBpThreads), 0, stream, b, d_tables, d_scratch);
  } else if (small)
    hipLaunchKernelGGL((crc32c_tiles_kernel<1, false>), dim3(blocks), dim3(kThreads), 0, stream, b, d_tables,
                       d_scratch, d_results);
  else
    hipLaunchKernelGGL((crc32c_tiles_kernel<4, false>), dim3(blocks), dim3(kThreads), 0, stream, b, d_tables,
                       d_scratch, d_results);
  hip_check(hipGetLastError(), "crc32c_tiles_kernel");
  hipLaunchKernelGGL(crc32c_fold_kernel, dim3(b.nseg), dim3(kThreads), 0, stream, b, d_tables, d_scratch, d_results);
  hip_check(hipGetLastError(), "crc32c_fold_kernel");
}

namespace {
std::mutex g_crc_opt_mu;
CrcLaunchOptions g_crc_opt;
}  // namespace

void set_crc_launch_options(const CrcLaunchOptions& o) {
  std::lock_guard<std::mutex> lk(g_crc_opt_mu);
  g_crc_opt = o;
}

CrcLaunchOptions crc_launch_options() {
  std::lock_guard<std::mutex> lk(g_crc_opt_mu);
  return g_crc_opt;
}

uint32_t* crc_scratch_alloc(uint64_t tiles) {
  uint32_t* p = nullptr;
  const size_t bytes = sizeof(uint32_t) * crc_scratch_words(tiles);
  hip_check(hipMalloc(reinterpret_cast<void**>(&p), bytes), "hipMalloc(crc scratch)");
  // all of it: callers carve per-slot scratches (each with its own header
  // counter) out of one allocation
  // hipMemset may still be running when it returns, and the kernels that use
  // this scratch go on non-blocking streams that do not order after it: wait
  hip_check(hipMemsetAsync(p, 0, bytes, nullptr), "hipMemsetAsync(crc scratch)");
  hip_check(hipStreamSynchronize(nullptr), "hipStreamSynchronize(crc scratch)");
  return p;
}

void launch_fill_pattern(uint8_t* dst, uint64_t n, uint64_t rot, uint64_t obj_off, hipStream_t stream) {
  if (n == 0) return;
  uint64_t groups = (n + 15) / 16;
  uint64_t blocks = (groups + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(fill_pattern_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream, dst, n, rot,
                     obj_off);
  hip_check(hipGetLastError(), "fill_pattern_kernel");
}

void launch_verify_pattern(const uint8_t* src, uint64_t n, uint64_t rot, uint64_t obj_off,
                           unsigned long long* d_count, unsigned long long* d_first, hipStream_t stream) {
  if (n == 0) return;
  uint64_t groups = (n + 15) / 16;
  uint64_t blocks = (groups + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(verify_pattern_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream, src, n, rot,
                     obj_off, d_count, d_first);
  hip_check(hipGetLastError(), "verify_pattern_kernel");
}

}  // namespace gcsb
