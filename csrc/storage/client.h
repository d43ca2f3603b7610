// Storage client: read / list / stat / write objects over HTTP (XML or JSON
// API) or gRPC (google.storage.v2.Storage), with the reference's retry policy.
//
// Reference: the benchmark builds a cloud.google.com/go/storage client either
// over HTTP/1.1 (CreateHttpClient, reference main.go:62-104) or gRPC with a
// connection pool of 1 (CreateGrpcClient, main.go:106-117), sets the retry
// policy (main.go:179-184) and reads objects with NewReader + io.Copy
// (main.go:134-140).  The client library itself is [lib]; its
// observable wire behaviour is reproduced here natively.
#pragma once
#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "core/util.h"
#include "net/socket.h"
#include "storage/auth.h"
#include "storage/retry.h"
#include "storage/sink.h"

namespace gcsb {


struct ClientConfig {
  std::string protocol = "http";  // http | http2 | grpc
  Endpoint endpoint;              // e.g. http://127.0.0.1:8080
  std::string http_api = "xml";   // xml (library default) | json (alt=media)
  std::string user_agent = "prince";  // reference user_agent_round_tripper wiring, main.go:100
  int max_conns_per_host = 100;       // reference main.go:31
  int max_idle_conns_per_host = 100;  // reference main.go:32
  int grpc_conn_pool_size = 1;        // reference main.go:30
  size_t read_chunk = 2 << 20;        // bytes per recv into the sink (reference intent, main.go:123-125)
  // HTTP/2 receive settings we advertise (gRPC and -client-protocol http2),
  // h2/h2_client.h H2ClientOptions: the largest DATA frame we accept (0 =
  // not advertised, the RFC 7540 default of 16,384 bytes grpc-go's client
  // leaves its peer with [lib]) and the stream / connection window (grpc-go's
  // BDP estimator stops at 16 MiB [lib]).  Defaults: the reference's.
  uint32_t h2_max_frame_size = 0;
  uint32_t h2_window = 16u << 20;
  // DATA frames up to this size are received many per recvmsg()
  // (H2DataCursor::read_spanning); 0 = one frame per receive (A/B)
  uint32_t h2_span_max_frame = 256u << 10;
  RetryPolicy retry;
  SocketOptions sock;
  std::shared_ptr<TokenSource> token;  // null = no Authorization header
  std::string project = "gcs-fuse-test";
  std::vector<int> cpus;  // transport/worker thread CPU set (empty = unpinned)
  // the HTTP/2 (gRPC) connection reader threads' CPU set (empty = cpus): a
  // multiplexed connection's one reader receives every stream's bytes, so it
  // gets a physical core the workers do not share (affinity.isolate_reader)
  std::vector<int> reader_cpus;
};

struct ObjectMeta {
  std::string name, bucket;
  int64_t size = 0, generation = 0, metageneration = 1;
  bool has_crc32c = false;
  uint32_t crc32c = 0;
  std::string md5;  // raw bytes
  std::string content_type;
  std::string updated;  // RFC3339
};

struct ReadResult {
  uint64_t bytes = 0;
  int attempts = 0;
  int64_t first_byte_ns = 0;  // steady clock, first body byte (TTFB)
  int64_t host_done_ns = 0;   // last byte received on the host
  ObjectInfo info;
  SinkResult sink;
  bool sink_begun = false;  // transport called sink.begin() (set by read_attempt)
  // Generation every attempt must read (0 = latest).  A retry/resume after a
  // partial read pins the generation the first attempt saw, as the storage
  // library's reader does, so the resumed bytes come from the same object
  // version; sliced reads pin the stat's generation for every slice.
  int64_t pin_generation = 0;
};

struct ListResult {
  std::vector<ObjectMeta> objects;
  std::vector<std::string> prefixes;
  std::string next_page_token;
};

// Bytes to upload. Implementations: host memory, GPU HBM staged through a
// pinned ring (csrc/gpu/engine.h).
class ByteSource {
 public:
  virtual ~ByteSource() = default;
  virtual uint64_t size() const = 0;
  // Next window of up to max bytes at the current offset; len 0 at end.
  virtual std::pair<const uint8_t*, size_t> next(size_t max) = 0;
  // Restart at `offset` (resumable upload recovery).
  virtual void seek(uint64_t offset) = 0;
  virtual bool has_crc32c() const { return false; }
  // The object's CRC32C (has_crc32c()); a source that checksums as it stages
  // (GpuByteSource) may have to finish that first when asked early.
  virtual uint32_t crc32c() const { return 0; }
  // crc32c() is known now, without waiting: a transport asks for it at the
  // start of an upload (StartResumableWrite / the session's metadata) only
  // then, and otherwise sends it with the last message / chunk.
  virtual bool crc32c_ready() const { return has_crc32c(); }
  // CRC32C of [off, off+len) when the source already holds it (the GPU
  // source checksums the object in HBM up front, chunk by chunk); false = the
  // caller computes it from the bytes.
  virtual bool range_crc32c(uint64_t off, size_t len, uint32_t* crc) {
    (void)off, (void)len, (void)crc;
    return false;
  }
  // The windows next() returns stay unchanged until the upload call returns
  // (no staging slot is refilled while the object is sent): the transport
  // may then hand their pages to the socket by reference (vmsplice + splice)
  // instead of copying them, since the final response proves the peer read
  // every byte.
  virtual bool stable_until_done() const { return false; }
};

class HostByteSource : public ByteSource {
 public:
  HostByteSource(const uint8_t* p, uint64_t n, bool compute_crc = true);
  uint64_t size() const override { return n_; }
  std::pair<const uint8_t*, size_t> next(size_t max) override;
  void seek(uint64_t off) override { off_ = off; }
  bool has_crc32c() const override { return has_crc_; }
  uint32_t crc32c() const override { return crc_; }
  bool stable_until_done() const override { return true; }  // the caller's buffer

 private:
  const uint8_t* p_;
  uint64_t n_, off_ = 0;
  bool has_crc_;
  uint32_t crc_ = 0;
};

struct WriteOptions {
  size_t chunk_bytes = 16 << 20;  // resumable chunk (library default 16 MiB) [lib]
  bool resumable = true;
  std::string content_type = "application/octet-stream";
};

struct CallStats {
  std::atomic<uint64_t> requests{0}, retries{0}, bytes_in{0}, bytes_out{0}, dials{0};
};

// Where an upload's time went (steady-clock ns from its start; 0 = not
// reached): the session's start RPC answered, the first and the last content
// byte handed to the socket, the final response.  Each upload fills its own
// and publishes it when it returns (StorageClient::last_upload): a client
// shared by uploading threads reports the last one to finish.
struct UploadPhases {
  int64_t start_rpc_ns = 0, first_send_ns = 0, last_send_ns = 0, response_ns = 0;
};

class StorageClient {
 public:
  virtual ~StorageClient() = default;
  // Full-object (limit<0) or ranged read into the sink, retried/resumed per
  // the retry policy. `cancel` aborts backoff sleeps.
  ReadResult read_object(const std::string& bucket, const std::string& object, Sink& sink, int64_t offset = 0,
                         int64_t limit = -1, const volatile bool* cancel = nullptr, int64_t generation = 0,
                         bool defer_finish = false);  // caller finishes the sink (overlaps its copy tail)
  ObjectMeta stat_object(const std::string& bucket, const std::string& object);
  // objects.compose / ComposeObject (1..32 sources, same bucket).
  ObjectMeta compose_object(const std::string& bucket, const std::string& dest, const std::vector<std::string>& sources,
                            const std::string& content_type = "");
  void delete_object(const std::string& bucket, const std::string& object);
  ListResult list_objects(const std::string& bucket, const std::string& prefix, int page_size = 1000,
                          const std::string& page_token = "", const std::string& delimiter = "");
  // Lists every page.
  std::vector<ObjectMeta> list_all(const std::string& bucket, const std::string& prefix, int page_size = 1000);
  ObjectMeta write_object(const std::string& bucket, const std::string& object, ByteSource& src,
                          const WriteOptions& opt = {});
  const ClientConfig& config() const { return cfg_; }
  CallStats& stats() { return stats_; }
  UploadPhases last_upload() const {
    std::lock_guard<std::mutex> lk(upload_mu_);
    return upload_;
  }
  virtual std::string transport_name() const = 0;
  // Network path actually used (gRPC: DirectPath vs CloudPath, see grpc_client.cc).
  virtual std::string transport_path() const { return "cloudpath"; }

 protected:
  void set_last_upload(const UploadPhases& p) {
    std::lock_guard<std::mutex> lk(upload_mu_);
    upload_ = p;
  }
  explicit StorageClient(ClientConfig cfg) : cfg_(std::move(cfg)) {}
  // One attempt; throws StorageError. `delivered` is incremented as bytes
  // are committed to the sink so the retry loop can resume.
  virtual void read_attempt(const std::string& bucket, const std::string& object, Sink& sink, int64_t offset,
                            int64_t limit, bool first_attempt, ReadResult* rr, uint64_t* delivered) = 0;
  virtual ObjectMeta stat_attempt(const std::string& bucket, const std::string& object) = 0;
  virtual ObjectMeta compose_attempt(const std::string& bucket, const std::string& dest,
                                     const std::vector<std::string>& sources, const std::string& content_type) = 0;
  virtual void delete_attempt(const std::string& bucket, const std::string& object) = 0;
  virtual ListResult list_attempt(const std::string& bucket, const std::string& prefix, int page_size,
                                  const std::string& page_token, const std::string& delimiter) = 0;
  virtual ObjectMeta write_impl(const std::string& bucket, const std::string& object, ByteSource& src,
                                const WriteOptions& opt) = 0;
  template <typename F>
  auto with_retry(F&& f, const volatile bool* cancel = nullptr) -> decltype(f());
  ClientConfig cfg_;
  CallStats stats_;

 private:
  mutable std::mutex upload_mu_;
  UploadPhases upload_;  // the last finished upload's (gRPC write_impl)
};

bool should_retry(const RetryPolicy& p, const StorageError& e, int attempt, int64_t t0);

template <typename F>
auto StorageClient::with_retry(F&& f, const volatile bool* cancel) -> decltype(f()) {
  Backoff bo(cfg_.retry);
  int64_t t0 = now_ns();
  for (int attempt = 1;; ++attempt) {
    try {
      ++stats_.requests;
      return f();
    } catch (const StorageError& e) {
      if (!should_retry(cfg_.retry, e, attempt, t0)) throw;
      ++stats_.retries;
      sleep_seconds(bo.pause(), cancel);
      if (cancel && *cancel) throw;
    }
  }
}

std::unique_ptr<StorageClient> make_http_client(const ClientConfig& cfg);
std::unique_ptr<StorageClient> make_grpc_client(const ClientConfig& cfg);
std::unique_ptr<StorageClient> make_client(const ClientConfig& cfg);  // dispatch on cfg.protocol

// x-goog-hash: "crc32c=<b64>,md5=<b64>" (may appear in several headers).
void parse_goog_hash(const std::string& value, bool* has_crc, uint32_t* crc, std::string* md5);
std::string format_goog_hash(uint32_t crc, const std::string& md5);
std::string crc32c_b64(uint32_t crc);
bool crc32c_from_b64(const std::string& b64, uint32_t* crc);

}  // namespace gcsb
