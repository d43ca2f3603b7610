// CDNA4 (gfx950) CRC32C kernels + synthetic-pattern fill/verify kernels.
// Design notes in crc32c_gpu.h and crc_types.h (tile geometry).  Wave64
// throughout: a wave owns a 16 KiB tile, read in 4 rounds of 4 KiB where lane
// l takes its own contiguous 64-byte chunk (4 x global_load_dwordx4; each
// 128-byte line is consumed by two lanes within 4 consecutive loads, so L1
// absorbs the 16 B-per-lane pattern).  The data has no reuse and never touches
// LDS; the LDS holds the 44 KiB of lookup tables: slice-by-16 (16 lookups per
// 16 B), one gap-shift table (a lane's state jumps 4032 B to its next chunk:
// 0.75 lookups per 16 B) and 6 wave-tree shift tables (1.5 per 16 B).
//
// Measured (profiles/r1_k1, scripts/crc_kernel_bench.py, 1 GiB in 32 MiB
// segments): round-0 kernel (4 KiB tiles, 16 B-strided lanes, 36 % of lookups
// spent on gap shifts) 2.4 TB/s -> lane-contiguous 256 B runs 3.0-3.1 TB/s
// (fewer lookups but L1-hostile 256 B lane strides) -> 64 B chunks in 4 KiB
// rounds 3.5-3.7 TB/s.  Random ds_read_b32 table lookups still cost ~4
// bank-conflict cycles per instruction; the conflict-free "nib" variant
// (nibble tables replicated per LDS bank, GCSB_CRC_K1=nib) removes them
// (0.16/instr) but doubles lookups and VALU and runs at 3.2 TB/s.
#include <hip/hip_runtime.h>

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

constexpr int kK1Threads = 512;                       // 8 waves (tiles) per workgroup: amortise the table fill
constexpr int kLdsWords = 16 * 256 + 7 * 4 * 256;     // slice16 + 6 tree + 1 gap shift tables = 11264 words (44 KiB)

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

__device__ __forceinline__ uint32_t mask_low_bytes(uint32_t w, int keep_from) {
  // zero bytes [0, keep_from) of a little-endian word (keep_from in 0..4)
  if (keep_from <= 0) return w;
  if (keep_from >= 4) return 0;
  return w & (0xFFFFFFFFu << (8 * keep_from));
}

// Lane `lane`'s 16 pieces of the tile starting at tstart, in CRC order:
// piece (k, j) = round k, chunk piece j at tstart + 4096 k + 64 lane + 16 j.
// Pieces before the segment start read as zeros (free for a raw CRC); the
// piece straddling it is masked.  Tiles are right-aligned to the segment end,
// so only the first tile of a segment has such a head.
__device__ __forceinline__ void load_lane_pieces(uint4 (&v)[kCrcRounds * kCrcChunkPieces], intptr_t tstart, int lane,
                                                 uintptr_t addr) {
#pragma unroll
  for (int k = 0; k < kCrcRounds; ++k)
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

// K1: raw CRC of every 4 KiB tile of every segment in the batch.
template <bool kK1LoadsFirst>
__global__ __launch_bounds__(kK1Threads) void crc32c_tiles_kernel(const CrcBatch b, const uint32_t* __restrict__ tabs,
                                                                   uint32_t* __restrict__ tile_out) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kLdsWords];
  {
    const uint4* src = reinterpret_cast<const uint4*>(tabs);
    uint4* dst = reinterpret_cast<uint4*>(s_tab);
#pragma unroll
    for (int i = threadIdx.x; i < kLdsWords / 4; i += kK1Threads) dst[i] = src[i];
  }
  __syncthreads();
  const uint32_t* sl = s_tab;
  const uint32_t* lane_shift = s_tab + 16 * 256;
  const int lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * (kK1Threads / 64);
  // gt only grows, so the segment search resumes where the last tile left it
  // (restarting from 0 cost up to kMaxSeg dependent scalar loads per tile)
  uint32_t s = 0;
  for (uint32_t gt = blockIdx.x * (kK1Threads / 64) + wave; gt < b.total_tiles; gt += nwaves) {
    while (s + 1 < b.nseg && b.seg[s + 1].tile_base <= gt) ++s;
    const uintptr_t addr = reinterpret_cast<uintptr_t>(b.seg[s].addr);
    const uint32_t len = b.seg[s].len;
    const uint32_t t = gt - b.seg[s].tile_base;
    const uintptr_t a16 = addr & ~uintptr_t(15);
    const uint64_t full = (addr + len - a16 + 15) / 16 - 1;
    const intptr_t vend = static_cast<intptr_t>(a16 + 16 * full);
    const intptr_t tstart = vend - static_cast<intptr_t>(kCrcTile) * static_cast<intptr_t>(b.seg[s].ntiles - t);
    uint4 v[kCrcRounds * kCrcChunkPieces];
    load_lane_pieces(v, tstart, lane, addr);
    // keep all 16 loads of the tile in flight before the first lookup (the
    // scheduler otherwise sinks them into the lookup chain: fewer bytes in
    // flight per wave)
    if (kK1LoadsFirst) __builtin_amdgcn_sched_barrier(0);
    uint32_t state = 0;
#pragma unroll
    for (int k = 0; k < kCrcRounds; ++k) {
      if (k) state = shift4(lane_shift + 6 * 1024, state);  // over the 4032-byte gap to this lane's next chunk
#pragma unroll
      for (int j = 0; j < kCrcChunkPieces; ++j) state = update16(sl, state, v[k * kCrcChunkPieces + j]);
    }
    // wave tree: lane l's last chunk ends 64 (63 - l) bytes before the tile end
#pragma unroll
    for (int lv = 0; lv < 6; ++lv) {
      const uint32_t other = __shfl_down(state, 1 << lv, 64);
      const uint32_t shifted = shift4(lane_shift + lv * 1024, state);
      if ((lane & ((2 << lv) - 1)) == 0) state = shifted ^ other;
    }
    if (lane == 0) tile_out[gt] = state;
  }
}

// K1, conflict-free variant ("nib"): the slice-by-16 lookups are split into
// 32 nibble tables (16 entries each) and the whole 2 KiB nibble set is
// replicated 32x in LDS so that lane l of each 32-lane LDS group reads only
// bank l: every lookup is one LDS cycle per group (random byte tables cost
// 2 + ~4 conflict cycles per wave instruction, profiles/r1_crc_pmc_*).  Twice
// the lookups (32 per 16 B) at a third of the cycles each; 88 KiB of LDS, so
// one 16-wave workgroup per CU.
constexpr int kK1NibThreads = 1024;
constexpr int kNibWords = 32 * 16 * 32;                  // 64 KiB replicated nibble tables
constexpr int kLdsNibWords = kNibWords + 7 * 4 * 256;    // + tree/gap shift tables = 92 KiB

__device__ __forceinline__ uint32_t nib_word(const uint32_t* __restrict__ lbase, uint32_t w, int t0) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) c ^= lbase[((t0 + j) * 16 + ((w >> (4 * j)) & 15)) * 32];
  return c;
}

__device__ __forceinline__ uint32_t update16_nib(const uint32_t* __restrict__ lbase, uint32_t state, uint4 v) {
  return nib_word(lbase, state ^ v.x, 0) ^ nib_word(lbase, v.y, 8) ^ nib_word(lbase, v.z, 16) ^
         nib_word(lbase, v.w, 24);
}

__global__ __launch_bounds__(kK1NibThreads) void crc32c_tiles_nib_kernel(const CrcBatch b,
                                                                         const CrcTables* __restrict__ tabs,
                                                                         uint32_t* __restrict__ tile_out) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kLdsNibWords];
  {
    const uint32_t* nib = &tabs->nib[0][0];
    for (int i = threadIdx.x; i < kNibWords; i += kK1NibThreads) s_tab[i] = nib[i >> 5];
    const uint4* src = reinterpret_cast<const uint4*>(&tabs->lane_shift[0][0][0]);
    uint4* dst = reinterpret_cast<uint4*>(s_tab + kNibWords);
    for (int i = threadIdx.x; i < 7 * 256; i += kK1NibThreads) dst[i] = src[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t* lbase = s_tab + (lane & 31);
  const uint32_t* lane_shift = s_tab + kNibWords;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * (kK1NibThreads / 64);
  uint32_t s = 0;
  for (uint32_t gt = blockIdx.x * (kK1NibThreads / 64) + wave; gt < b.total_tiles; gt += nwaves) {
    while (s + 1 < b.nseg && b.seg[s + 1].tile_base <= gt) ++s;
    const uintptr_t addr = reinterpret_cast<uintptr_t>(b.seg[s].addr);
    const uint32_t len = b.seg[s].len;
    const uint32_t t = gt - b.seg[s].tile_base;
    const uintptr_t a16 = addr & ~uintptr_t(15);
    const uint64_t full = (addr + len - a16 + 15) / 16 - 1;
    const intptr_t vend = static_cast<intptr_t>(a16 + 16 * full);
    const intptr_t tstart = vend - static_cast<intptr_t>(kCrcTile) * static_cast<intptr_t>(b.seg[s].ntiles - t);
    uint4 v[kCrcRounds * kCrcChunkPieces];
    load_lane_pieces(v, tstart, lane, addr);
    uint32_t state = 0;
#pragma unroll
    for (int k = 0; k < kCrcRounds; ++k) {
      if (k) state = shift4(lane_shift + 6 * 1024, state);
#pragma unroll
      for (int j = 0; j < kCrcChunkPieces; ++j) state = update16_nib(lbase, state, v[k * kCrcChunkPieces + j]);
    }
#pragma unroll
    for (int lv = 0; lv < 6; ++lv) {
      const uint32_t other = __shfl_down(state, 1 << lv, 64);
      const uint32_t shifted = shift4(lane_shift + lv * 1024, state);
      if ((lane & ((2 << lv) - 1)) == 0) state = shifted ^ other;
    }
    if (lane == 0) tile_out[gt] = state;
  }
}

// K2: fold tiles -> segment raw CRC, add the tail, fixup, compare.
__global__ __launch_bounds__(256) void crc32c_segments_kernel(const CrcBatch b, const CrcTables* __restrict__ t,
                                                              const uint32_t* __restrict__ tiles,
                                                              CrcSegResult* __restrict__ out) {
  const uint32_t s = blockIdx.x;
  if (s >= b.nseg) return;
  const uint32_t T = b.seg[s].ntiles;
  const uint32_t base = b.seg[s].tile_base;
  const int k = threadIdx.x;
  const int lane = k & 63;
  uint32_t acc = 0;
  const int M = static_cast<int>((T + 255) >> 8);
  for (int m = M - 1; m >= 0; --m) {
    acc = shift4(&t->tile_shift[8][0][0], acc);
    const uint32_t j = static_cast<uint32_t>(k) + 256u * static_cast<uint32_t>(m);
    if (j < T) acc ^= tiles[base + T - 1 - j];
  }
#pragma unroll
  for (int lv = 0; lv < 6; ++lv) {
    const uint32_t other = __shfl_down(acc, 1 << lv, 64);
    if ((lane & ((2 << lv) - 1)) == 0) acc ^= shift4(&t->tile_shift[lv][0][0], other);
  }
  __shared__ uint32_t part[4];
  if (lane == 0) part[k >> 6] = acc;
  __syncthreads();
  if (k == 0) {
    const uint32_t v0 = part[0] ^ shift4(&t->tile_shift[6][0][0], part[1]);
    const uint32_t v2 = part[2] ^ shift4(&t->tile_shift[6][0][0], part[3]);
    uint32_t raw = v0 ^ shift4(&t->tile_shift[7][0][0], v2);
    const uint32_t len = b.seg[s].len;
    if (len > 0) {
      const uintptr_t addr = reinterpret_cast<uintptr_t>(b.seg[s].addr);
      const uintptr_t a16 = addr & ~uintptr_t(15);
      const uintptr_t e = addr + len;
      const uintptr_t vend = a16 + 16 * ((e - a16 + 15) / 16 - 1);
      const uint8_t* p = reinterpret_cast<const uint8_t*>(vend > addr ? vend : addr);
      const uint8_t* pe = reinterpret_cast<const uint8_t*>(e);
      for (; p < pe; ++p) raw = (raw >> 8) ^ t->slice16[0][(raw ^ *p) & 0xff];
    }
    const uint32_t crc = raw ^ b.seg[s].fixup;
    CrcSegResult r;
    r.raw = raw;
    r.crc = crc;
    r.status = (b.seg[s].flags & 1) ? (crc == b.seg[s].expected ? 1u : 2u) : 0u;
    r.pad = 0;
    out[s] = r;
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

enum class K1Variant { kSlice16, kNib };

// GCSB_CRC_K1=slice16|nib selects the tile kernel (A/B switch; default below).
K1Variant k1_variant() {
  static K1Variant v = [] {
    const char* e = std::getenv("GCSB_CRC_K1");
    if (e && std::string(e) == "slice16") return K1Variant::kSlice16;
    if (e && std::string(e) == "nib") return K1Variant::kNib;
    return K1Variant::kSlice16;
  }();
  return v;
}

// GCSB_K1_LOADS_FIRST=0 lets the scheduler interleave the tile loads with the
// lookups (A/B switch; default: all 16 loads issued first).
bool k1_loads_first() {
  static bool v = [] {
    const char* e = std::getenv("GCSB_K1_LOADS_FIRST");
    return !(e && *e == '0');
  }();
  return v;
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

void launch_crc32c_batch(const CrcBatch& b, const CrcTables* d_tables, uint32_t* d_tile_scratch,
                         CrcSegResult* d_results, hipStream_t stream) {
  if (b.nseg == 0) return;
  if (b.total_tiles > 0) {
    if (k1_variant() == K1Variant::kNib) {
      constexpr uint32_t tiles_per_block = kK1NibThreads / 64;
      uint32_t blocks = (b.total_tiles + tiles_per_block - 1) / tiles_per_block;
      if (blocks > 256) blocks = 256;  // one 88 KiB workgroup per CU, grid-stride over tiles
      hipLaunchKernelGGL(crc32c_tiles_nib_kernel, dim3(blocks), dim3(kK1NibThreads), 0, stream, b, d_tables,
                         d_tile_scratch);
      hip_check(hipGetLastError(), "crc32c_tiles_nib_kernel");
    } else {
      constexpr uint32_t tiles_per_block = kK1Threads / 64;
      uint32_t blocks = (b.total_tiles + tiles_per_block - 1) / tiles_per_block;
      if (blocks > 1024) blocks = 1024;
      if (k1_loads_first())
        hipLaunchKernelGGL(crc32c_tiles_kernel<true>, dim3(blocks), dim3(kK1Threads), 0, stream, b,
                           reinterpret_cast<const uint32_t*>(d_tables), d_tile_scratch);
      else
        hipLaunchKernelGGL(crc32c_tiles_kernel<false>, dim3(blocks), dim3(kK1Threads), 0, stream, b,
                           reinterpret_cast<const uint32_t*>(d_tables), d_tile_scratch);
      hip_check(hipGetLastError(), "crc32c_tiles_kernel");
    }
  }
  hipLaunchKernelGGL(crc32c_segments_kernel, dim3(b.nseg), dim3(256), 0, stream, b, d_tables, d_tile_scratch,
                     d_results);
  hip_check(hipGetLastError(), "crc32c_segments_kernel");
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
