// Synthetic GCS endpoint: HTTP/1.1 (XML + JSON media, JSON metadata/list,
// resumable/simple uploads, OAuth token + metadata-server token endpoints) and
// h2c gRPC (google.storage.v2.Storage) on ONE loopback port, sniffed by the
// connection preface.  Fault injection covers the failure classes the
// reference's retry policy exists for (reference main.go:179-184): 429/503
// bursts, mid-stream disconnects, corrupted bytes (CRC failures), slow drip.
#pragma once
#include <atomic>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "h2/h2.h"
#include "net/socket.h"
#include "server/store.h"

namespace gcsb {

struct FaultConfig {
  std::atomic<int> fail_next{0};            // fail the next N data requests...
  std::atomic<int> fail_status{503};        // ...with this HTTP status (gRPC: mapped code)
  std::atomic<int64_t> disconnect_at{-1};   // cut the connection after this many body bytes...
  std::atomic<int> disconnect_count{0};     // ...this many times
  std::atomic<int64_t> corrupt_at{-1};      // flip one byte at this object offset...
  std::atomic<int> corrupt_count{0};        // ...in this many responses
  std::atomic<int64_t> throttle_bps{0};     // per-response rate cap (bytes/s), 0 = none
  std::atomic<int> latency_ms{0};           // added time-to-first-byte
  std::atomic<int> drop_trailers_count{0};  // gRPC: cut the connection after the last DATA, before trailers
  std::atomic<int64_t> stall_at{-1};        // pause a response this long before sending this object offset...
  std::atomic<int> stall_ms{0};
  std::atomic<int> stall_count{0};          // ...in this many responses (client read-timeout tests)
  std::atomic<int> finalize_delay_ms{0};    // gRPC WriteObject: hold the final response this long
};

struct ServerConfig {
  std::string host = "127.0.0.1";
  int port = 0;  // 0 = ephemeral
  bool require_auth = false;
  std::string jwt_public_key_pem;  // verify JWT assertions at /token if set
  uint64_t grpc_chunk = 2 << 20;   // ReadObjectResponse content bytes per message (reference main.go:123-124)
  int sndbuf = 0;          // 0 = kernel autotuning (an explicit size disables it)
  bool zero_copy = true;   // synthetic object bodies by page reference (no user-space copy)
  // ...from the pattern's THP copy by vmsplice + splice (default), or, false,
  // by sendfile() from its memfd (rounds 1-3; also the fallback when THP
  // memory cannot be had): profiles/r3_splice/thp_source
  bool send_vmsplice = true;
  std::vector<int> cpus;   // pin connection/handler threads (empty = unpinned)
  // gRPC connections' send-scheduler threads (empty = cpus): one core of
  // their own, off the multiplexed reader's and the workers' cores
  std::vector<int> send_cpus;
  // WriteObject CRC32C workers (empty = cpus): a core apart from the
  // connection thread that receives the upload
  std::vector<int> crc_cpus;
  // HTTP/2: DATA frame cap while several streams share a connection
  // (H2Writer::set_quantum and the send scheduler's turn; 0 = a whole
  // message per turn).  ReadObject messages are <= 2 MiB and the scheduler
  // already serves streams round-robin a message at a time: 256 KiB frames
  // cost the 48-stream block 15-30% with no better tail (profiles/r4_main6).
  // A new read's first frame sent ahead of the queue did not lower its TTFB
  // either: at 48 streams the ~2 ms before a read's first byte is the
  // connection's bytes in flight in the socket buffers, not the endpoint's
  // queue (profiles/r4_main7 mux; endpoint request -> HEADERS 10-30 us).
  size_t h2_quantum = 0;
  // Attribution A/B only: false = WriteObject messages are not CRC-checked
  // (the endpoint trusts the client's per-message crc32c), so nothing but
  // the receive reads the uploaded bytes.  Default true.
  bool write_verify = true;
  // https / gRPC over TLS (ALPN h2 or http/1.1) when both are set (PEM files)
  std::string tls_cert_file, tls_key_file;
};

struct ServerStats {
  std::atomic<uint64_t> connections{0}, http_requests{0}, grpc_calls{0}, bytes_sent{0}, bytes_received{0},
      faults_injected{0}, auth_failures{0};
  // WriteObject content receives on the connection thread (recv calls and
  // bytes): the upload's receive granularity
  std::atomic<uint64_t> write_recvs{0}, write_recv_bytes{0};
  // object-body sends (HTTP GET bodies, gRPC ReadObject streams): the
  // kernel's send chronographs over each (TCP_INFO deltas, us) and the
  // congestion window at its end -- what bounded the endpoint's sending
  std::atomic<uint64_t> body_sends{0}, body_wall_us{0}, tcp_busy_us{0}, tcp_rwnd_limited_us{0},
      tcp_sndbuf_limited_us{0}, tcp_cwnd_bytes_sum{0};
  // account one body send on fd that started at t0_ns with chronographs a
  void note_body_send(int fd, const TcpChrono& a, bool a_ok, int64_t t0_ns);
  // HTTP/2 DATA frames sent and how long their stream handlers queued for
  // the connection (FIFO, H2Writer): the endpoint's fairness across streams
  H2SendStats h2_send;
  // a stream's request complete (END_STREAM seen) -> its response HEADERS
  // written: the endpoint's share of a read's TTFB
  std::atomic<uint64_t> h2_responses{0}, h2_ttfb_ns{0}, h2_ttfb_max_ns{0};
  void note_ttfb(int64_t ns);
};
// bodies at least this long get their send chronographs read
constexpr uint64_t kChronoMinBody = 8u << 20;

class FakeGcsServer {
 public:
  FakeGcsServer(ServerConfig cfg, std::shared_ptr<ObjectStore> store);
  ~FakeGcsServer();
  void start();
  void stop();
  int port() const { return port_; }
  std::string url() const {
    return std::string(tls_ctx_ ? "https://" : "http://") + cfg_.host + ":" + std::to_string(port_);
  }
  ObjectStore& store() { return *store_; }
  FaultConfig& faults() { return faults_; }
  ServerStats& stats() { return stats_; }
  const ServerConfig& config() const { return cfg_; }
  // Tokens issued by /token and the metadata endpoint (checked when require_auth).
  std::string issue_token();
  bool token_valid(const std::string& tok);

  // Connection handlers (server_http1.cc / server_grpc.cc).
  void serve_http1(std::unique_ptr<class BufferedConn> bc);
  void serve_h2(std::unique_ptr<class BufferedConn> bc);

 private:
  void accept_loop();
  void handle_conn(int fd);
  ServerConfig cfg_;
  std::shared_ptr<ObjectStore> store_;
  FaultConfig faults_;
  ServerStats stats_;
  std::unique_ptr<Listener> listener_;
  void* tls_ctx_ = nullptr;  // SSL_CTX when serving TLS
  int port_ = 0;
  std::thread accept_thread_;
  std::atomic<bool> stopping_{false};
  std::mutex conns_mu_;
  std::set<int> conn_fds_;
  std::vector<std::thread> conn_threads_;
  std::atomic<int> live_threads_{0};
  std::mutex tok_mu_;
  std::set<std::string> tokens_;
  uint64_t tok_seq_ = 0;
};

}  // namespace gcsb
