// Object store of the synthetic GCS server.
//
// The reference benchmarks a real bucket (reference main.go:44,52: bucket
// "princer-working-dirs", objects "princer_100M_files/file_<id>").  Neither GCS
// nor the network exists on the build or GPU boxes, so every benchmark runs
// against this loopback server.  Synthetic objects are virtual slices of the
// shared pattern (csrc/core/content.h) with precomputed CRC32C/MD5; uploaded
// objects are stored as real bytes.
#pragma once
#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <tuple>
#include <string>
#include <vector>

#include "core/crc32c.h"

namespace gcsb {

// Bytes of an uploaded object: anonymous mmap advised for transparent huge
// pages and grown by doubling with mremap, so a 64 MiB upload takes ~32 page
// faults instead of 16384 (first-touch faults dominated the fake server's
// upload cost) and growth never copies.
class Blob {
 public:
  Blob() = default;
  ~Blob();
  Blob(const Blob&) = delete;
  Blob& operator=(const Blob&) = delete;
  Blob(Blob&& o) noexcept { swap(o); }
  Blob& operator=(Blob&& o) noexcept {
    Blob t(std::move(o));
    swap(t);
    return *this;
  }
  void reserve(size_t n);
  void append(const void* p, size_t n);
  // Grows by n bytes and returns a pointer to them (caller fills them).
  uint8_t* extend(size_t n);
  void clear() { size_ = 0; }
  size_t size() const { return size_; }
  const uint8_t* data() const { return p_; }

 private:
  void swap(Blob& o) noexcept {
    std::swap(p_, o.p_);
    std::swap(size_, o.size_);
    std::swap(cap_, o.cap_);
  }
  uint8_t* p_ = nullptr;
  size_t size_ = 0, cap_ = 0;
};

struct StoredObject {
  std::string bucket, name;
  uint64_t size = 0;
  int64_t generation = 0;
  int64_t metageneration = 1;
  int64_t created_us = 0;
  std::string content_type = "application/octet-stream";
  bool synthetic = false;
  bool hollow = false;  // upload whose bytes the server did not retain (metadata only)
  uint64_t rot = 0;                                  // synthetic: pattern rotation
  std::shared_ptr<const Blob> data;                  // uploaded objects
  uint32_t crc32c = 0;
  // MD5 (raw 16 bytes, empty if disabled) is computed on first use: an
  // upload's timed path must not pay for a digest only metadata reads need.
  const std::string& md5() const;
  void set_md5(std::string m) { md5_ = std::move(m); md5_lazy_ = false; }
  void set_md5_lazy() { md5_lazy_ = true; }
  // False while a lazy MD5 has not been computed yet (upload responses then
  // omit it instead of computing it inside the client's timed upload).
  bool md5_ready() const { return !md5_lazy_ || md5_done_.load(std::memory_order_acquire); }

  // Contiguous bytes [off, off+n) with n <= kPatternExt.
  const uint8_t* bytes(uint64_t off, uint64_t n) const;
  // Synthetic objects: (fd, file offset) of [off, off+n) for sendfile(); false otherwise.
  bool file_range(uint64_t off, int* fd, uint64_t* foff) const;
  // Synthetic objects sent by vmsplice (PatternBuffer::send_by_vmsplice):
  // [off, off+n) (n <= kPatternExt) in the pattern's THP copy; nullptr
  // otherwise (then file_range / bytes).
  const uint8_t* splice_bytes(uint64_t off, uint64_t n) const;
  uint32_t crc32c_range(uint64_t off, uint64_t n) const;

 private:
  mutable std::once_flag md5_once_;
  mutable std::string md5_;
  mutable std::atomic<bool> md5_done_{false};
  bool md5_lazy_ = false;
};

struct UploadSession {
  std::string id, bucket, name, content_type;
  Blob data;
  uint32_t data_crc = 0;  // running CRC32C of the received bytes
  uint64_t received = 0;  // persisted size
  bool retain = true;     // false: verify (size, CRC32C) and drop the bytes
  int64_t expected_size = -1;
  void append(const void* p, size_t n) {
    if (retain) data.append(p, n);
    data_crc = crc32c_extend(data_crc, p, n);
    received += n;
  }
  // Same, with the bytes' CRC32C already computed by the caller.
  void append_with_crc(const void* p, size_t n, uint32_t crc) {
    if (retain) data.append(p, n);
    data_crc = crc32c_combine(data_crc, crc, n);
    received += n;
  }
  bool has_crc = false;
  uint32_t crc = 0;
  bool finalized = false;
  std::shared_ptr<const StoredObject> result;
  std::mutex mu;
};

class ObjectStore {
 public:
  explicit ObjectStore(bool compute_md5 = true) : compute_md5_(compute_md5) {}
  // Upload benchmarking: verify size + CRC32C of uploads but keep only their
  // metadata (the server-side analogue of the reference's io.Discard sink).
  void set_retain_uploads(bool r) { retain_uploads_ = r; }
  bool retain_uploads() const { return retain_uploads_; }
  std::shared_ptr<const StoredObject> get(const std::string& bucket, const std::string& name) const;
  std::shared_ptr<const StoredObject> add_synthetic(const std::string& bucket, const std::string& name, uint64_t size);
  // Adds count objects prefix<i>suffix, computing checksums in parallel.
  void add_synthetic_range(const std::string& bucket, const std::string& prefix, const std::string& suffix,
                           int first, int count, uint64_t size);
  std::shared_ptr<const StoredObject> put(const std::string& bucket, const std::string& name,
                                          Blob data, const std::string& content_type,
                                          const uint32_t* known_crc = nullptr);
  bool remove(const std::string& bucket, const std::string& name);
  // objects.compose / ComposeObject: dest = concatenation of 1..32 sources.
  // CRC32C is the GF(2) combine of the sources' CRCs, so metadata-only
  // (non-retained) sources compose without bytes; the result keeps bytes
  // only if every source has them and uploads are retained.
  std::shared_ptr<const StoredObject> compose(const std::string& bucket, const std::string& dest,
                                              const std::vector<std::string>& sources,
                                              const std::string& content_type, std::string* err);
  // Objects with the prefix, sorted by name, names > start_after, at most max.
  std::vector<std::shared_ptr<const StoredObject>> list(const std::string& bucket, const std::string& prefix,
                                                        const std::string& start_after, size_t max) const;
  size_t count() const;

  std::shared_ptr<UploadSession> start_upload(const std::string& bucket, const std::string& name,
                                              const std::string& content_type, int64_t expected_size);
  std::shared_ptr<UploadSession> find_upload(const std::string& id) const;
  // Finalizes a session; verifies the client-supplied crc32c if any.
  std::shared_ptr<const StoredObject> finalize_upload(UploadSession& s, std::string* err);

  // Chunk CRCs for gRPC ReadObject messages aligned at multiples of `chunk`
  // from offset 0 (cached per object).
  uint32_t chunk_crc(const StoredObject& o, uint64_t off, uint64_t n, uint64_t chunk) const;

 private:
  int64_t next_generation();
  bool compute_md5_;
  bool retain_uploads_ = true;
  mutable std::shared_mutex mu_;
  std::map<std::pair<std::string, std::string>, std::shared_ptr<const StoredObject>> objects_;
  mutable std::mutex up_mu_;
  std::map<std::string, std::shared_ptr<UploadSession>> uploads_;
  mutable std::mutex crc_mu_;
  mutable std::map<std::tuple<std::string, std::string, int64_t, uint64_t>, std::shared_ptr<std::vector<uint32_t>>>
      chunk_crcs_;
  int64_t last_gen_ = 0;
  std::mutex gen_mu_;
  uint64_t upload_seq_ = 0;
};

}  // namespace gcsb
