#include "net/socket.h"

#include <atomic>

#include <arpa/inet.h>
#include <fcntl.h>
#include <sys/uio.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <poll.h>
#include <signal.h>
#include <sys/sendfile.h>
#include <linux/sockios.h>
#include <sys/ioctl.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <map>
#include <algorithm>
#include <mutex>
#include <vector>

#include "core/util.h"

namespace gcsb {

namespace {
// sendfile() and writev() have no MSG_NOSIGNAL: a peer that closed its end
// (a client's read timeout, a cancelled stream) would kill the whole process
// with SIGPIPE.  Like other network runtimes (Go ignores it on sockets), turn
// it into EPIPE -- unless the host program installed a handler of its own.
// (Python already ignores SIGPIPE; the C++ tools and tests do not.)
struct IgnoreSigpipe {
  IgnoreSigpipe() {
    struct sigaction cur {};
    if (::sigaction(SIGPIPE, nullptr, &cur) == 0 && cur.sa_handler == SIG_DFL) ::signal(SIGPIPE, SIG_IGN);
  }
} g_ignore_sigpipe;
}  // namespace

Endpoint Endpoint::parse(const std::string& url) {
  Endpoint ep;
  std::string rest = url;
  size_t p = rest.find("://");
  if (p != std::string::npos) {
    ep.scheme = to_lower(rest.substr(0, p));
    rest = rest.substr(p + 3);
  }
  ep.port = ep.scheme == "https" ? 443 : 80;
  size_t slash = rest.find('/');
  std::string hostport = rest.substr(0, slash);
  if (slash != std::string::npos) {
    ep.base_path = rest.substr(slash);
    while (!ep.base_path.empty() && ep.base_path.back() == '/') ep.base_path.pop_back();
  }
  size_t colon = hostport.rfind(':');
  if (colon != std::string::npos && hostport.find(']') == std::string::npos) {
    ep.host = hostport.substr(0, colon);
    ep.port = std::stoi(hostport.substr(colon + 1));
  } else {
    ep.host = hostport;
  }
  if (ep.host.empty()) ep.host = "127.0.0.1";
  return ep;
}

std::string Endpoint::host_header() const {
  bool dflt = (scheme == "http" && port == 80) || (scheme == "https" && port == 443);
  return dflt ? host : host + ":" + std::to_string(port);
}

void apply_socket_options(int fd, const SocketOptions& opt) {
  int one = 1;
  if (opt.nodelay) setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  if (opt.rcvbuf > 0) setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &opt.rcvbuf, sizeof(opt.rcvbuf));
  if (opt.sndbuf > 0) setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &opt.sndbuf, sizeof(opt.sndbuf));
  if (!opt.congestion.empty())
    (void)setsockopt(fd, IPPROTO_TCP, TCP_CONGESTION, opt.congestion.data(),
                     static_cast<socklen_t>(opt.congestion.size()));
  if (opt.loopback_rto_min) set_loopback_rto_min(fd);
  if (opt.io_timeout_ms > 0) {
    timeval tv{opt.io_timeout_ms / 1000, (opt.io_timeout_ms % 1000) * 1000};
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  }
}

static SSL_CTX* client_ssl_ctx(bool verify, const std::string& ca_file) {
  static std::mutex mu;
  static std::map<std::pair<bool, std::string>, SSL_CTX*> ctx;
  std::lock_guard<std::mutex> lk(mu);
  SSL_CTX*& c = ctx[{verify, ca_file}];
  if (!c) {
    c = SSL_CTX_new(TLS_client_method());
    SSL_CTX_set_min_proto_version(c, TLS1_2_VERSION);
    if (verify) {
      if (!ca_file.empty()) {
        if (SSL_CTX_load_verify_locations(c, ca_file.c_str(), nullptr) != 1)
          throw StorageError("TLS: cannot load CA file " + ca_file, false);
      } else {
        SSL_CTX_set_default_verify_paths(c);
      }
      SSL_CTX_set_verify(c, SSL_VERIFY_PEER, nullptr);
    } else {
      SSL_CTX_set_verify(c, SSL_VERIFY_NONE, nullptr);
    }
  }
  return c;
}

static std::string alpn_wire(const std::string& protos) {  // "h2,http/1.1" -> length-prefixed list
  std::string w;
  size_t b = 0;
  while (b <= protos.size()) {
    size_t e = protos.find(',', b);
    if (e == std::string::npos) e = protos.size();
    if (e > b) {
      w.push_back(static_cast<char>(e - b));
      w.append(protos, b, e - b);
    }
    b = e + 1;
  }
  return w;
}

void* make_server_tls_ctx(const TlsServer& t) {
  SSL_CTX* c = SSL_CTX_new(TLS_server_method());
  if (!c) throw std::runtime_error("SSL_CTX_new failed");
  if (SSL_CTX_use_certificate_chain_file(c, t.cert_file.c_str()) != 1 ||
      SSL_CTX_use_PrivateKey_file(c, t.key_file.c_str(), SSL_FILETYPE_PEM) != 1) {
    SSL_CTX_free(c);
    throw std::runtime_error("TLS: cannot load server certificate/key " + t.cert_file + " / " + t.key_file);
  }
  SSL_CTX_set_alpn_select_cb(
      c,
      [](SSL*, const unsigned char** out, unsigned char* outlen, const unsigned char* in, unsigned int inlen,
         void*) -> int {
        // prefer h2, then http/1.1
        for (const char* want : {"h2", "http/1.1"}) {
          const size_t wl = std::strlen(want);
          for (unsigned int i = 0; i < inlen;) {
            unsigned int l = in[i];
            if (l == wl && i + 1 + l <= inlen && std::memcmp(in + i + 1, want, l) == 0) {
              *out = in + i + 1;
              *outlen = static_cast<unsigned char>(l);
              return SSL_TLSEXT_ERR_OK;
            }
            i += 1 + l;
          }
        }
        return SSL_TLSEXT_ERR_NOACK;
      },
      nullptr);
  return c;
}

void free_server_tls_ctx(void* ctx) {
  if (ctx) SSL_CTX_free(static_cast<SSL_CTX*>(ctx));
}

std::string Conn::alpn() const {
  if (!ssl_) return "";
  const unsigned char* p = nullptr;
  unsigned int n = 0;
  SSL_get0_alpn_selected(ssl_, &p, &n);
  return p ? std::string(reinterpret_cast<const char*>(p), n) : "";
}

int reserve_fd_table(int slots) {
  static std::once_flag once;
  static int reserved = 0;
  std::call_once(once, [slots] {
    rlimit rl{};
    if (getrlimit(RLIMIT_NOFILE, &rl) != 0) return;
    const rlim_t want = static_cast<rlim_t>(slots);
    if (rl.rlim_cur < want && rl.rlim_max > rl.rlim_cur) {
      rlimit up = rl;
      up.rlim_cur = std::min<rlim_t>(rl.rlim_max, want);
      if (setrlimit(RLIMIT_NOFILE, &up) == 0) rl = up;
    }
    const int top = static_cast<int>(std::min<rlim_t>(rl.rlim_cur, want)) - 1;
    if (top < 64) return;
    const int fd = ::open("/dev/null", O_RDONLY | O_CLOEXEC);
    if (fd < 0) return;
    // F_DUPFD takes the lowest free number >= top: the table grows to hold it
    // (and never shrinks), and no descriptor in use is touched
    const int hi = ::fcntl(fd, F_DUPFD_CLOEXEC, top);
    if (hi >= 0) {
      ::close(hi);
      reserved = top + 1;
    }
    ::close(fd);
  });
  return reserved;
}

std::unique_ptr<Conn> Conn::dial(const Endpoint& ep, const SocketOptions& opt) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  std::string port = std::to_string(ep.port);
  int rc = getaddrinfo(ep.host.c_str(), port.c_str(), &hints, &res);
  if (rc != 0) throw StorageError("resolve " + ep.host + ": " + gai_strerror(rc), true);
  int fd = -1;
  std::string last_err;
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    apply_socket_options(fd, opt);
    // non-blocking connect with timeout
    int fl = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, fl | O_NONBLOCK);
    int c = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (c != 0 && errno == EINPROGRESS) {
      pollfd pfd{fd, POLLOUT, 0};
      int pr = ::poll(&pfd, 1, opt.connect_timeout_ms > 0 ? opt.connect_timeout_ms : -1);
      int soerr = 0;
      socklen_t sl = sizeof(soerr);
      if (pr == 1) getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl);
      c = (pr == 1 && soerr == 0) ? 0 : -1;
      if (pr == 0) errno = ETIMEDOUT;
      else if (soerr) errno = soerr;
    }
    if (c == 0) {
      fcntl(fd, F_SETFL, fl);
      break;
    }
    last_err = std::strerror(errno);
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) throw StorageError("connect " + ep.host + ":" + port + ": " + last_err, true);
  auto conn = std::make_unique<Conn>();
  conn->fd_ = fd;
  conn->fill_bytes_ = opt.fill_bytes;
  if (ep.scheme == "https") {
    SSL* ssl = SSL_new(client_ssl_ctx(opt.tls_verify, opt.tls_ca_file));
    SSL_set_fd(ssl, fd);
    SSL_set_tlsext_host_name(ssl, ep.host.c_str());
    if (opt.tls_verify) SSL_set1_host(ssl, ep.host.c_str());  // host-name check of the leaf certificate
    if (!opt.alpn.empty()) {
      std::string w = alpn_wire(opt.alpn);
      SSL_set_alpn_protos(ssl, reinterpret_cast<const unsigned char*>(w.data()), static_cast<unsigned>(w.size()));
    }
    if (SSL_connect(ssl) != 1) {
      long vr = SSL_get_verify_result(ssl);
      std::string why = vr != X509_V_OK ? std::string(": certificate ") + X509_verify_cert_error_string(vr) : "";
      SSL_free(ssl);
      conn->fd_ = fd;  // closed by ~Conn
      conn->fill_bytes_ = opt.fill_bytes;
      // a certificate failure will not fix itself: not retryable
      throw StorageError("TLS handshake with " + ep.host + " failed" + why, vr == X509_V_OK);
    }
    conn->ssl_ = ssl;
    conn->io_timeout_ms_ = opt.io_timeout_ms;
    conn->tls_nonblocking();
  }
  return conn;
}

std::unique_ptr<Conn> Conn::adopt_tls(int fd, const SocketOptions& opt, void* ssl_ctx) {
  auto conn = adopt(fd, opt);
  if (!ssl_ctx) return conn;
  SSL* ssl = SSL_new(static_cast<SSL_CTX*>(ssl_ctx));
  SSL_set_fd(ssl, fd);
  if (SSL_accept(ssl) != 1) {
    SSL_free(ssl);
    throw StorageError("TLS accept failed", false);
  }
  conn->ssl_ = ssl;
  conn->io_timeout_ms_ = opt.io_timeout_ms;
  conn->tls_nonblocking();
  return conn;
}

void Conn::tls_nonblocking() {
  int fl = fcntl(fd_, F_GETFL, 0);
  fcntl(fd_, F_SETFL, fl | O_NONBLOCK);
}

// Waits (without ssl_mu_) until the socket is ready for what SSL asked for.
void Conn::wait_ready(int ssl_err) {
  pollfd pfd{fd_, static_cast<short>(ssl_err == SSL_ERROR_WANT_WRITE ? POLLOUT : POLLIN), 0};
  for (;;) {
    int pr = ::poll(&pfd, 1, io_timeout_ms_ > 0 ? io_timeout_ms_ : -1);
    if (pr > 0) return;
    if (pr == 0) throw StorageError(ssl_err == SSL_ERROR_WANT_WRITE ? "write timeout" : "read timeout", true);
    if (errno != EINTR) throw StorageError(std::string("poll: ") + std::strerror(errno), true);
  }
}

// One SSL_read / SSL_write under ssl_mu_; returns > 0 bytes, 0 = clean EOF (read).
int Conn::ssl_io(bool write, void* buf, size_t n) {
  const int len = static_cast<int>(n > (1u << 30) ? (1u << 30) : n);
  for (;;) {
    int k, e;
    {
      std::lock_guard<std::mutex> lk(ssl_mu_);
      if (!ssl_) throw StorageError("TLS connection closed", true);
      ERR_clear_error();
      k = write ? SSL_write(ssl_, buf, len) : SSL_read(ssl_, buf, len);
      e = k > 0 ? SSL_ERROR_NONE : SSL_get_error(ssl_, k);
    }
    if (k > 0) return k;
    if (e == SSL_ERROR_ZERO_RETURN && !write) return 0;
    if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) {
      wait_ready(e);
      continue;
    }
    if (e == SSL_ERROR_SYSCALL && errno == EINTR) continue;
    throw StorageError(write ? "TLS write error" : "TLS read error", true);
  }
}

std::unique_ptr<Conn> Conn::adopt(int fd, const SocketOptions& opt) {
  apply_socket_options(fd, opt);
  auto conn = std::make_unique<Conn>();
  conn->fd_ = fd;
  conn->fill_bytes_ = opt.fill_bytes;
  return conn;
}

Conn::~Conn() { close(); }

void Conn::close() {
  for (int& p : pipe_)
    if (p >= 0) {
      ::close(p);
      p = -1;
    }
  if (ssl_) {
    std::lock_guard<std::mutex> lk(ssl_mu_);
    SSL_shutdown(ssl_);  // best effort on the non-blocking socket
    SSL_free(ssl_);
    ssl_ = nullptr;
  }
  if (fd_ >= 0) {
    ::close(fd_);
    fd_ = -1;
  }
}

void Conn::shutdown_write() {
  if (fd_ >= 0) ::shutdown(fd_, SHUT_WR);
}

std::atomic<uint64_t> g_recv_calls{0}, g_recv_bytes{0};
std::atomic<uint64_t> g_diag_calls{0}, g_diag_empty{0}, g_diag_short{0}, g_diag_inq{0}, g_diag_want{0}, g_diag_ns{0};

RecvStats recv_stats() {
  RecvStats r;
  r.calls = g_recv_calls.load();
  r.bytes = g_recv_bytes.load();
  r.diag_calls = g_diag_calls.load();
  r.diag_empty = g_diag_empty.load();
  r.diag_short = g_diag_short.load();
  r.diag_inq_bytes = g_diag_inq.load();
  r.diag_want_bytes = g_diag_want.load();
  r.diag_recv_ns = g_diag_ns.load();
  return r;
}

size_t Conn::read_some(void* buf, size_t n) {
  if (fd_ < 0) throw StorageError("read on closed connection", true);
  for (;;) {
    ssize_t r;
    if (ssl_) {
      r = ssl_io(false, buf, n);
    } else {
      static const bool diag = [] {
        const char* e = std::getenv("GCSB_RECV_DIAG");
        return e && e[0] == '1';
      }();
      int64_t t0 = 0;
      if (diag && n >= (64u << 10)) {
        int inq = 0;
        if (::ioctl(fd_, SIOCINQ, &inq) == 0) {
          g_diag_calls.fetch_add(1, std::memory_order_relaxed);
          g_diag_want.fetch_add(n, std::memory_order_relaxed);
          g_diag_inq.fetch_add(static_cast<uint64_t>(inq), std::memory_order_relaxed);
          if (inq == 0) g_diag_empty.fetch_add(1, std::memory_order_relaxed);
          else if (static_cast<size_t>(inq) < n) g_diag_short.fetch_add(1, std::memory_order_relaxed);
          t0 = now_ns();
        }
      }
      r = ::recv(fd_, buf, n, 0);
      if (t0) g_diag_ns.fetch_add(static_cast<uint64_t>(now_ns() - t0), std::memory_order_relaxed);
    }
    if (r >= 0) {
      bytes_read_ += static_cast<uint64_t>(r);
      g_recv_calls.fetch_add(1, std::memory_order_relaxed);
      g_recv_bytes.fetch_add(static_cast<uint64_t>(r), std::memory_order_relaxed);
      return static_cast<size_t>(r);
    }
    if (errno == EINTR) continue;
    if (errno == EAGAIN || errno == EWOULDBLOCK) throw StorageError("read timeout", true);
    throw StorageError(std::string("recv: ") + std::strerror(errno), true);
  }
}

size_t Conn::read_somev(struct iovec* iov, int cnt) {
  if (ssl_ || cnt == 1) return read_some(iov[0].iov_base, iov[0].iov_len);
  if (fd_ < 0) throw StorageError("read on closed connection", true);
  for (;;) {
    msghdr m{};
    m.msg_iov = iov;
    m.msg_iovlen = static_cast<size_t>(cnt);
    const ssize_t r = ::recvmsg(fd_, &m, 0);
    if (r >= 0) {
      bytes_read_ += static_cast<uint64_t>(r);
      g_recv_calls.fetch_add(1, std::memory_order_relaxed);
      g_recv_bytes.fetch_add(static_cast<uint64_t>(r), std::memory_order_relaxed);
      return static_cast<size_t>(r);
    }
    if (errno == EINTR) continue;
    if (errno == EAGAIN || errno == EWOULDBLOCK) throw StorageError("read timeout", true);
    throw StorageError(std::string("recv: ") + std::strerror(errno), true);
  }
}

void Conn::read_exact(void* buf, size_t n) {
  auto* p = static_cast<uint8_t*>(buf);
  while (n > 0) {
    size_t r;
    if (!ssl_) {
      ssize_t k = ::recv(fd_, p, n, MSG_WAITALL);
      if (k < 0) {
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) throw StorageError("read timeout", true);
        throw StorageError(std::string("recv: ") + std::strerror(errno), true);
      }
      r = static_cast<size_t>(k);
      bytes_read_ += r;
    } else {
      r = read_some(p, n);
    }
    if (r == 0) throw StorageError("unexpected EOF", true);
    p += r;
    n -= r;
  }
}

void Conn::write_all(const void* buf, size_t n) {
  iovec iov{const_cast<void*>(buf), n};
  writev_all(&iov, 1);
}

void Conn::writev_all(struct iovec* iov, int cnt, bool more) {
  if (fd_ < 0) throw StorageError("write on closed connection", true);
  if (ssl_) {
    for (int i = 0; i < cnt; ++i) {
      auto* p = static_cast<const uint8_t*>(iov[i].iov_base);
      size_t n = iov[i].iov_len;
      while (n > 0) {
        int k = ssl_io(true, const_cast<uint8_t*>(p), n);
        p += k;
        n -= static_cast<size_t>(k);
        bytes_written_ += static_cast<uint64_t>(k);
      }
    }
    return;
  }
  while (cnt > 0) {
    msghdr msg{};
    msg.msg_iov = iov;
    msg.msg_iovlen = static_cast<size_t>(cnt > 1024 ? 1024 : cnt);
    ssize_t w = ::sendmsg(fd_, &msg, MSG_NOSIGNAL | (more ? MSG_MORE : 0));
    if (w < 0) {
      if (errno == EINTR) continue;
      throw StorageError(std::string("send: ") + std::strerror(errno), true);
    }
    bytes_written_ += static_cast<uint64_t>(w);
    size_t left = static_cast<size_t>(w);
    while (cnt > 0 && left >= iov->iov_len) {
      left -= iov->iov_len;
      ++iov;
      --cnt;
    }
    if (cnt > 0 && left) {
      iov->iov_base = static_cast<uint8_t*>(iov->iov_base) + left;
      iov->iov_len -= left;
    }
  }
}

void Conn::ensure_pipe() {
  if (pipe_[0] >= 0) return;
  if (::pipe2(pipe_, O_CLOEXEC) != 0) throw StorageError(std::string("pipe2: ") + std::strerror(errno), false);
  // a 1 MiB pipe (fs.pipe-max-size default): 2 syscalls per MiB
  (void)::fcntl(pipe_[1], F_SETPIPE_SZ, 1 << 20);
  const int c = ::fcntl(pipe_[1], F_GETPIPE_SZ);
  pipe_cap_ = c > 0 ? static_cast<size_t>(c) : 65536;
}

void Conn::splice_out(size_t left, bool more) {
  while (left > 0) {
    const unsigned fl = SPLICE_F_MOVE | (more ? SPLICE_F_MORE : 0u);
    ssize_t w = ::splice(pipe_[0], nullptr, fd_, nullptr, left, fl);
    if (w < 0) {
      if (errno == EINTR) continue;
      const int e = errno;
      // the pipe may still hold page references: drop it with the connection
      for (int& q : pipe_) {
        ::close(q);
        q = -1;
      }
      throw StorageError(std::string("splice: ") + std::strerror(e), true);
    }
    if (w == 0) throw StorageError("splice: connection closed", true);
    bytes_written_ += static_cast<uint64_t>(w);
    left -= static_cast<size_t>(w);
  }
}

void Conn::splice_user_all(const void* data, size_t n, bool more) {
  if (fd_ < 0) throw StorageError("write on closed connection", true);
  if (ssl_) return write_all(data, n);
  ensure_pipe();
  auto* p = static_cast<const uint8_t*>(data);
  while (n > 0) {
    iovec iov{const_cast<uint8_t*>(p), std::min(n, pipe_cap_)};
    ssize_t k = ::vmsplice(pipe_[1], &iov, 1, 0);
    if (k < 0) {
      if (errno == EINTR) continue;
      throw StorageError(std::string("vmsplice: ") + std::strerror(errno), true);
    }
    p += k;
    n -= static_cast<size_t>(k);
    splice_out(static_cast<size_t>(k), more || n > 0);
  }
}

void Conn::sendfile_all(int in_fd, uint64_t off, size_t n, bool more) {
  if (fd_ < 0) throw StorageError("write on closed connection", true);
  if (ssl_) {  // no kernel TLS here: fall back to pread + SSL_write
    std::vector<uint8_t> buf(std::min<size_t>(n, 1 << 20));
    while (n > 0) {
      ssize_t r = ::pread(in_fd, buf.data(), std::min(n, buf.size()), static_cast<off_t>(off));
      if (r <= 0) throw StorageError("pread for TLS send failed", true);
      write_all(buf.data(), static_cast<size_t>(r));
      off += static_cast<uint64_t>(r);
      n -= static_cast<size_t>(r);
    }
    return;
  }
  if (more) {
    int one = 1;
    setsockopt(fd_, IPPROTO_TCP, TCP_CORK, &one, sizeof(one));
  }
  off_t o = static_cast<off_t>(off);
  while (n > 0) {
    ssize_t w = ::sendfile(fd_, in_fd, &o, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw StorageError(std::string("sendfile: ") + std::strerror(errno), true);
    }
    if (w == 0) throw StorageError("sendfile: source ended", false);
    bytes_written_ += static_cast<uint64_t>(w);
    n -= static_cast<size_t>(w);
  }
  if (more) {
    int zero = 0;
    setsockopt(fd_, IPPROTO_TCP, TCP_CORK, &zero, sizeof(zero));
  }
}

Listener::Listener(const std::string& host, int port, int backlog) {
  int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) throw std::runtime_error("socket failed");
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  if (inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
    std::string err = std::strerror(errno);
    ::close(fd);
    throw std::runtime_error("bind " + host + ":" + std::to_string(port) + ": " + err);
  }
  // The endpoint's congestion control goes on the LISTENING socket, so an
  // accepted connection starts with it.  Set after accept() (round 3) the
  // child had already run the host default's init: BBR's marks the socket
  // for internal pacing (sk_pacing_status), which no later TCP_CONGESTION
  // undoes, so "cubic" connections were still paced by an hrtimer per
  // 64 KiB skb -- ~4,000 timer interrupts per 256 MiB read on the sending
  // and receiving cores, whose count moved every block's rate
  // (profiles/r4_recvcost).
  set_endpoint_congestion_control(fd);
  if (::listen(fd, backlog) != 0) {
    ::close(fd);
    throw std::runtime_error("listen failed");
  }
  socklen_t sl = sizeof(addr);
  getsockname(fd, reinterpret_cast<sockaddr*>(&addr), &sl);
  port_ = ntohs(addr.sin_port);
  fd_ = fd;
}

Listener::~Listener() {
  close();
  int fd = fd_.exchange(-1);
  if (fd >= 0) ::close(fd);
}

int Listener::accept_fd() {
  for (;;) {
    if (closed_.load(std::memory_order_acquire)) return -1;
    int c = ::accept4(fd_.load(std::memory_order_relaxed), nullptr, nullptr, SOCK_CLOEXEC);
    if (c >= 0) {
      if (closed_.load(std::memory_order_acquire)) {
        ::close(c);
        return -1;
      }
      return c;
    }
    if (errno == EINTR || errno == ECONNABORTED) continue;
    return -1;
  }
}

// Wakes a blocked accept_fd() (shutdown) without releasing the descriptor:
// the fd number cannot be reused under a concurrent accept4; the destructor
// closes it once the accepting thread is gone.
void Listener::close() {
  if (!closed_.exchange(true, std::memory_order_acq_rel)) {
    int fd = fd_.load(std::memory_order_relaxed);
    if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
  }
}

}  // namespace gcsb
