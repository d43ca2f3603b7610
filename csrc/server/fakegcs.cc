#include "server/fakegcs.h"

#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>

#include "core/affinity.h"
#include "core/content.h"
#include "core/util.h"
#include "net/buffered.h"

namespace gcsb {

void ServerStats::note_ttfb(int64_t ns) {
  const uint64_t v = ns > 0 ? static_cast<uint64_t>(ns) : 0;
  h2_responses.fetch_add(1, std::memory_order_relaxed);
  h2_ttfb_ns.fetch_add(v, std::memory_order_relaxed);
  uint64_t m = h2_ttfb_max_ns.load(std::memory_order_relaxed);
  while (v > m && !h2_ttfb_max_ns.compare_exchange_weak(m, v, std::memory_order_relaxed)) {
  }
}

void ServerStats::note_body_send(int fd, const TcpChrono& a, bool a_ok, int64_t t0_ns) {
  TcpChrono b;
  if (!a_ok || !read_tcp_chrono(fd, &b)) return;
  ++body_sends;
  body_wall_us += static_cast<uint64_t>((now_ns() - t0_ns) / 1000);
  tcp_busy_us += b.busy_us - a.busy_us;
  tcp_rwnd_limited_us += b.rwnd_limited_us - a.rwnd_limited_us;
  tcp_sndbuf_limited_us += b.sndbuf_limited_us - a.sndbuf_limited_us;
  tcp_cwnd_bytes_sum += b.cwnd_bytes;
}

FakeGcsServer::FakeGcsServer(ServerConfig cfg, std::shared_ptr<ObjectStore> store)
    : cfg_(std::move(cfg)), store_(std::move(store)) {}

FakeGcsServer::~FakeGcsServer() {
  stop();
  free_server_tls_ctx(tls_ctx_);
}

void FakeGcsServer::start() {
  reserve_fd_table();
  // build the pattern buffer (+ its THP copy for vmsplice, or its memfd for
  // sendfile) before the first request, so no read pays for it
  //
  // The memfd's page cache lands on the NUMA node of the thread that writes
  // it; every served byte is read from there by the send path and copied by
  // the client's receive thread.  Build it on a thread pinned to the
  // endpoint's CPUs (the rank's GPU-local node), not on whichever node the
  // caller (the Python main thread) happens to run.
  // The THP send source (PatternBuffer::thp, the default) is placed the
  // same way: by first touch on the pinned builder thread.
  if (cfg_.zero_copy) {
    const bool send_vmsplice = cfg_.send_vmsplice;
    auto build = [send_vmsplice] {
      if (!send_vmsplice || !PatternBuffer::instance().thp()) PatternBuffer::instance().memfd();
    };
    if (cfg_.cpus.empty()) {
      build();
    } else {
      std::thread([this, &build] {
        pin_current_thread(cfg_.cpus);
        bind_numa_node(current_numa_node());
        build();
        bind_numa_node(-1);
      }).join();
    }
  }
  if (!cfg_.tls_cert_file.empty() && !tls_ctx_) {
    TlsServer t;
    t.cert_file = cfg_.tls_cert_file;
    t.key_file = cfg_.tls_key_file;
    tls_ctx_ = make_server_tls_ctx(t);
  }
  listener_ = std::make_unique<Listener>(cfg_.host, cfg_.port);
  port_ = listener_->port();
  stopping_ = false;
  accept_thread_ = std::thread([this] { accept_loop(); });
}

void FakeGcsServer::stop() {
  if (!listener_) return;
  stopping_ = true;
  listener_->close();
  if (accept_thread_.joinable()) accept_thread_.join();
  {
    std::lock_guard<std::mutex> lk(conns_mu_);
    for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
  }
  // connection threads are detached; wait for them to drain
  for (int i = 0; i < 5000 && live_threads_.load() > 0; ++i)
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  listener_.reset();
}

void FakeGcsServer::accept_loop() {
  name_current_thread("gcsb-srv-accept");
  for (;;) {
    int fd = listener_->accept_fd();
    if (fd < 0) break;
    if (stopping_) {
      ::close(fd);
      break;
    }
    ++stats_.connections;
    {
      std::lock_guard<std::mutex> lk(conns_mu_);
      conn_fds_.insert(fd);
    }
    ++live_threads_;
    std::thread([this, fd] {
      pin_current_thread(cfg_.cpus);
      name_current_thread("gcsb-srv-conn");
      try {
        handle_conn(fd);
      } catch (...) {
      }
      {
        std::lock_guard<std::mutex> lk(conns_mu_);
        conn_fds_.erase(fd);
      }
      --live_threads_;
    }).detach();
  }
}

void FakeGcsServer::handle_conn(int fd) {
  SocketOptions so;
  so.sndbuf = cfg_.sndbuf;
  set_endpoint_congestion_control(fd);
  so.rcvbuf = 0;
  if (tls_ctx_) {
    // TLS: the protocol comes from ALPN (h2 = gRPC, else HTTP/1.1)
    auto c = Conn::adopt_tls(fd, so, tls_ctx_);
    const bool h2 = c->alpn() == "h2";
    auto bc = std::make_unique<BufferedConn>(std::move(c));
    if (h2)
      serve_h2(std::move(bc));
    else
      serve_http1(std::move(bc));
    return;
  }
  auto bc = std::make_unique<BufferedConn>(Conn::adopt(fd, so));
  char peek[3];
  ssize_t k = 0;
  for (int tries = 0; tries < 1000; ++tries) {
    k = ::recv(fd, peek, 3, MSG_PEEK | MSG_WAITALL);
    if (k == 3 || k <= 0) break;
  }
  if (k != 3) return;
  if (std::memcmp(peek, "PRI", 3) == 0)
    serve_h2(std::move(bc));
  else
    serve_http1(std::move(bc));
}

std::string FakeGcsServer::issue_token() {
  std::lock_guard<std::mutex> lk(tok_mu_);
  std::string t = "ya29.fake-" + std::to_string(++tok_seq_) + "-" + std::to_string(wall_ns() % 100000007);
  tokens_.insert(t);
  return t;
}

bool FakeGcsServer::token_valid(const std::string& tok) {
  std::lock_guard<std::mutex> lk(tok_mu_);
  return tokens_.count(tok) > 0;
}

}  // namespace gcsb
