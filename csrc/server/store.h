// Object store of the synthetic GCS server.
//
// The reference benchmarks a real bucket (reference main.go:44,52: bucket
// "princer-working-dirs", objects "princer_100M_files/file_<id>").  Neither GCS
// nor the network exists on the build or GPU boxes, so every benchmark runs
// against this loopback server.  Synthetic objects are virtual slices of the
// shared pattern (csrc/core/content.h) with precomputed CRC32C/MD5; uploaded
// objects are stored as real bytes.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <tuple>
#include <string>
#include <vector>

namespace gcsb {

struct StoredObject {
  std::string bucket, name;
  uint64_t size = 0;
  int64_t generation = 0;
  int64_t metageneration = 1;
  int64_t created_us = 0;
  std::string content_type = "application/octet-stream";
  bool synthetic = false;
  uint64_t rot = 0;                                  // synthetic: pattern rotation
  std::shared_ptr<const std::vector<uint8_t>> data;  // uploaded objects
  uint32_t crc32c = 0;
  std::string md5;  // raw 16 bytes, empty if not computed

  // Contiguous bytes [off, off+n) with n <= kPatternExt.
  const uint8_t* bytes(uint64_t off, uint64_t n) const;
  // Synthetic objects: (fd, file offset) of [off, off+n) for sendfile(); false otherwise.
  bool file_range(uint64_t off, int* fd, uint64_t* foff) const;
  uint32_t crc32c_range(uint64_t off, uint64_t n) const;
};

struct UploadSession {
  std::string id, bucket, name, content_type;
  std::vector<uint8_t> data;
  int64_t expected_size = -1;
  bool has_crc = false;
  uint32_t crc = 0;
  bool finalized = false;
  std::shared_ptr<const StoredObject> result;
  std::mutex mu;
};

class ObjectStore {
 public:
  explicit ObjectStore(bool compute_md5 = true) : compute_md5_(compute_md5) {}
  std::shared_ptr<const StoredObject> get(const std::string& bucket, const std::string& name) const;
  std::shared_ptr<const StoredObject> add_synthetic(const std::string& bucket, const std::string& name, uint64_t size);
  // Adds count objects prefix<i>suffix, computing checksums in parallel.
  void add_synthetic_range(const std::string& bucket, const std::string& prefix, const std::string& suffix,
                           int first, int count, uint64_t size);
  std::shared_ptr<const StoredObject> put(const std::string& bucket, const std::string& name,
                                          std::vector<uint8_t> data, const std::string& content_type);
  bool remove(const std::string& bucket, const std::string& name);
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
