// Blocking TCP connections (optionally TLS via OpenSSL) used by every
// transport.  One connection is owned by one thread at a time, except the
// HTTP/2 client where a reader thread owns recv and writers serialize send.
//
// Reference counterpart: Go net/http's Transport dials/keeps-alive TCP(+TLS)
// connections (reference main.go:65-73); grpc-go dials one HTTP/2 connection
// per pool entry (main.go:30,111).
#pragma once
#include <atomic>
#include <sys/types.h>
#include <sys/uio.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>

typedef struct ssl_st SSL;
typedef struct ssl_ctx_st SSL_CTX;

namespace gcsb {

struct Endpoint {
  std::string scheme = "http";  // http | https
  std::string host = "127.0.0.1";
  int port = 80;
  std::string base_path;  // path prefix, e.g. "" or "/storage"
  static Endpoint parse(const std::string& url);
  std::string host_header() const;
};

struct SocketOptions {
  int rcvbuf = 0;  // 0 = kernel autotuning
  int sndbuf = 0;
  bool nodelay = true;
  int connect_timeout_ms = 10000;
  int io_timeout_ms = 0;  // 0 = none (reference: http.Client.Timeout=0, main.go:94)
  // https endpoints: verify the server certificate chain and host name
  // against the system roots (or tls_ca_file); ALPN protocol to offer
  // ("h2" for gRPC, "http/1.1" for the HTTP client).
  bool tls_verify = true;
  std::string tls_ca_file;
  std::string alpn;
  // TCP congestion control of client sockets, set before connect() so the
  // connection never runs the host default's init ("" = host default).
  // BBR (the GPU boxes' default) marks a socket for internal pacing: on a
  // loopback link every 64 KiB skb of an upload then waits on an hrtimer
  // (profiles/r4_recvcost).
  std::string congestion;
  // Loopback endpoints only: minimum RTO kLoopbackRtoMinUs instead of 200 ms
  // (set_loopback_rto_min); never for a real network path.
  bool loopback_rto_min = false;
  // Most bytes one fill (or refill) of the reader's small-read buffer takes
  // from the socket (<= its 16 KiB).  A fill for a 9-byte frame header also
  // takes the payload behind it, which then costs a second copy out of the
  // buffer: up to 16 KiB per message, 1.6% of a 1 MiB read.
  size_t fill_bytes = 16384;
};

// Server-side TLS context from PEM files (fake GCS endpoint over https);
// ALPN selects "h2" when offered, else "http/1.1".
struct TlsServer {
  std::string cert_file, key_file;
};

// Process-wide count of Conn::read_some calls (one recv() each) and their
// bytes: the average receive size of a read path (diagnostics).
struct RecvStats {
  uint64_t calls = 0, bytes = 0;
  // GCSB_RECV_DIAG=1: for reads of >= 64 KiB (payload into a sink), the
  // socket's queue (SIOCINQ) just before the recv(): empty (the call
  // blocks: the receiver outran its sender), short (less than asked), and
  // the queued bytes.  One extra syscall per read, diagnostics only.
  uint64_t diag_calls = 0, diag_empty = 0, diag_short = 0, diag_inq_bytes = 0, diag_want_bytes = 0;
  uint64_t diag_recv_ns = 0;  // wall time inside those recv() calls
};
RecvStats recv_stats();

// Grow the process's file-descriptor table to `slots` entries once, now.
// The kernel doubles the table when an fd number outgrows it, and in a
// multi-threaded process each growth waits out an RCU grace period while
// every other thread's socket()/accept() sleeps behind it: a 48-worker run
// dialing its last connections stalled ~150 ms at once (profiles/r3_w48_tail:
// threads in D state, wait channel expand_files).  Raises the soft
// RLIMIT_NOFILE toward `slots` when the hard limit allows.  Returns the
// table size reserved (0 if nothing was done).
int reserve_fd_table(int slots = 8192);

class Conn {
 public:
  Conn() = default;
  ~Conn();
  Conn(const Conn&) = delete;
  Conn& operator=(const Conn&) = delete;

  static std::unique_ptr<Conn> dial(const Endpoint& ep, const SocketOptions& opt);
  static std::unique_ptr<Conn> adopt(int fd, const SocketOptions& opt);
  // Server side of a TLS connection (handshake done here); nullptr ctx = plain.
  static std::unique_ptr<Conn> adopt_tls(int fd, const SocketOptions& opt, void* ssl_ctx);
  // Negotiated ALPN protocol ("" if none / plain TCP).
  std::string alpn() const;

  // Returns bytes read (0 = orderly EOF); throws StorageError(retryable) on reset.
  size_t read_some(void* buf, size_t n);
  // One recvmsg() into iov[0..cnt) in order (plain TCP; TLS: iov[0] alone).
  size_t read_somev(struct iovec* iov, int cnt);
  // Reads exactly n bytes or throws (EOF mid-way is a retryable error).
  void read_exact(void* buf, size_t n);
  void write_all(const void* buf, size_t n);
  void writev_all(struct iovec* iov, int cnt, bool more = false);
  // Zero-copy send of a file range (sendfile); `more` corks for a following write.
  void sendfile_all(int in_fd, uint64_t off, size_t n, bool more = false);
  // Zero-copy send of user memory: vmsplice() its pages into a pipe, splice()
  // the pipe into the socket.  The socket buffers then REFERENCE the pages, so
  // the caller must leave them unchanged until the peer has read the bytes
  // (for an upload: until its final response).  TLS falls back to a copy.
  void splice_user_all(const void* p, size_t n, bool more = false);
  void shutdown_write();
  void close();
  int fd() const { return fd_; }
  bool is_open() const { return fd_ >= 0; }
  bool tls() const { return ssl_ != nullptr; }
  uint64_t bytes_read() const { return bytes_read_; }
  size_t fill_bytes() const { return fill_bytes_; }
  uint64_t bytes_written() const { return bytes_written_; }

 private:
  // TLS: an SSL object must not be entered by two threads at once, but an
  // HTTP/2 connection reads on one thread while others write.  After the
  // handshake the socket is non-blocking; each SSL_read / SSL_write runs under
  // ssl_mu_ and the thread waits for readiness (poll) without holding it.
  int ssl_io(bool write, void* buf, size_t n);
  void wait_ready(int ssl_err);
  void tls_nonblocking();
  int fd_ = -1;
  SSL* ssl_ = nullptr;
  std::mutex ssl_mu_;
  int io_timeout_ms_ = 0;
  size_t fill_bytes_ = 16384;
  uint64_t bytes_read_ = 0;
  uint64_t bytes_written_ = 0;
  void ensure_pipe();
  void splice_out(size_t n, bool more);  // the pipe's first n bytes to the socket
  int pipe_[2] = {-1, -1};  // splice_user_all's page pipe (lazily created)
  size_t pipe_cap_ = 0;
};

// Listening socket for the synthetic server.
class Listener {
 public:
  explicit Listener(const std::string& host, int port, int backlog = 1024);
  ~Listener();
  int port() const { return port_; }
  int fd() const { return fd_.load(std::memory_order_relaxed); }
  // Returns -1 when closed.
  int accept_fd();
  void close();

 private:
  std::atomic<int> fd_{-1};
  std::atomic<bool> closed_{false};
  int port_ = 0;
};

void apply_socket_options(int fd, const SocketOptions& opt);
// The kernel's per-connection send chronographs (TCP_INFO): microseconds the
// sender was busy, limited by the peer's receive window, or limited by its
// own send buffer; plus the congestion window in bytes.  false if the kernel
// does not report them.
struct TcpChrono {
  uint64_t busy_us = 0, rwnd_limited_us = 0, sndbuf_limited_us = 0;
  uint64_t cwnd_bytes = 0;
};
bool read_tcp_chrono(int fd, TcpChrono* out);
// The synthetic endpoint's congestion control on its connections
// (GCSB_SRV_CC; default "cubic", "default" = the host's).  The GPU boxes
// default to BBR, whose paced window on a loopback link held the endpoint's
// congestion window at 2.3-3.8 MiB and cost the one-stream HTTP read 20-35%
// (cubic: 7.9-9.7 MiB, profiles/r3_twins/cc).  An unprivileged process may
// pick any algorithm in net.ipv4.tcp_allowed_congestion_control; a refusal
// leaves the host's default.  The `ceiling` probe's sender uses it too.
// The synthetic endpoint's sockets (listener first, so accepted sockets
// inherit it): the congestion control (GCSB_SRV_CC, default cubic) and a
// loopback-sized minimum retransmission timeout.  The default 200 ms RTO
// min turns one receive-queue drop into a 200+ ms read (one 256 MiB HTTP
// read of 16 ms took 226 ms, profiles/r4_main8); on loopback the RTT is
// microseconds.
constexpr int kLoopbackRtoMinUs = 5000;
void set_loopback_rto_min(int fd);
void set_endpoint_congestion_control(int fd);
const std::string& endpoint_congestion_control();
// SSL_CTX for a TLS server (throws on bad cert/key); owned by the caller (free_server_tls_ctx).
void* make_server_tls_ctx(const TlsServer& t);
void free_server_tls_ctx(void* ctx);

}  // namespace gcsb
