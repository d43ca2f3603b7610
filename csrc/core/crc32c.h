// CRC32C (Castagnoli) — host implementation and GF(2) combine algebra.
//
// The reference never computes a checksum itself: the Go storage library
// (cloud.google.com/go/storage v1.33.0, reference go.mod:6) checks CRC32C of
// every full HTTP read against `x-goog-hash` and gRPC carries a crc32c per
// `ChecksummedData` message.  Here the same algebra is shared by
// the host path (SSE4.2 `crc32` instruction), the synthetic server, and the
// CDNA4 kernels in csrc/gpu/crc32c_kernels.hip, which get their lookup tables
// from the builders below so host and device agree bit for bit.
//
// Terminology used throughout the code base:
//   raw(d)      CRC register after processing d from state 0, no final xor.
//               raw is GF(2)-linear in d and unaffected by leading zero bytes.
//   shift(s,n)  register s advanced over n zero bytes = s * x^(8n) mod P.
//   crc32c(d) = shift(~0, |d|) ^ raw(d) ^ ~0 = raw(d) ^ fixup(|d|).
#pragma once
#include <cstddef>
#include <cstdint>

namespace gcsb {

constexpr uint32_t kCrc32cPoly = 0x82F63B78u;  // reflected 0x1EDC6F41

// Standard CRC32C of a buffer ("123456789" -> 0xE3069283).
uint32_t crc32c(const void* data, size_t n);
// Continue a standard CRC32C: crc32c(a||b) == crc32c_extend(crc32c(a), b).
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
// Linear register update: returns shift(state, n) ^ raw(data).
uint32_t crc32c_raw_update(uint32_t state, const void* data, size_t n);

// GF(2)[x] / P arithmetic in the reflected bit order.
uint32_t gf2_multmodp(uint32_t a, uint32_t b);
// x^(8n) mod P.
uint32_t crc32c_x8n(uint64_t nbytes);
// state advanced over n zero bytes.
uint32_t crc32c_shift(uint32_t state, uint64_t nbytes);
// crc32c(A||B) from crc32c(A), crc32c(B), |B|.
uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
// crc32c(d) == raw(d) ^ crc32c_fixup(|d|).
uint32_t crc32c_fixup(uint64_t nbytes);

// Table builders used by the GPU engine (uploaded once per device).
// slice[k][b] = raw of byte b followed by k zero bytes  (slice-by-16).
void crc32c_build_slice16(uint32_t slice[16][256]);
// tab[j][b] = shift(b << 8j, n): shift(s, n) = tab0[s&ff]^tab1[s>>8&ff]^...
void crc32c_build_shift_table(uint64_t nbytes, uint32_t tab[4][256]);
// Apply a shift table on the host (mirror of the device lookup).
uint32_t crc32c_apply_shift_table(const uint32_t tab[4][256], uint32_t s);

// Hardware capability (SSE4.2) detected at runtime.
bool crc32c_hw_available();

}  // namespace gcsb
