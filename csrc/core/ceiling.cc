#include "core/ceiling.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <string>
#include <thread>

#include "core/affinity.h"
#include "core/hugebuf.h"
#include "net/socket.h"

namespace gcsb {

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double thread_cpu_s() {
  rusage ru{};
  getrusage(RUSAGE_THREAD, &ru);
  return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}

[[noreturn]] void fail(const char* what) {
  throw std::runtime_error(std::string("ceiling: ") + what + ": " + std::strerror(errno));
}

// An anonymous page-locked (when allowed) ring, faulted in by the caller.
struct Ring {
  uint8_t* p = nullptr;
  size_t n = 0;
  Ring(size_t bytes, int pages) : n(bytes) {
    void* m = ::mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) fail("mmap(ring)");
    if (pages == 1) (void)madvise(m, n, MADV_HUGEPAGE);
    if (pages == 2) (void)madvise(m, n, MADV_NOHUGEPAGE);
    (void)mlock(m, n);
    std::memset(m, 0, n);
    p = static_cast<uint8_t*>(m);
  }
  ~Ring() {
    if (p) ::munmap(p, n);
  }
};

struct Fd {
  int fd = -1;
  explicit Fd(int f = -1) : fd(f) {}
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
  Fd(const Fd&) = delete;
  Fd& operator=(const Fd&) = delete;
};

double median(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

}  // namespace

CeilingResult memcpy_ceiling(const CeilingConfig& c) {
  CeilingResult res;
  std::exception_ptr err;
  // a thread of its own: pinning must not leak into the caller
  std::thread t([&] {
    try {
      pin_current_thread(c.recv_cpus);
      std::vector<uint8_t> src(c.object_bytes);
      for (size_t i = 0; i < src.size(); i += 4096) src[i] = static_cast<uint8_t>(i >> 12);
      Ring ring(c.ring_bytes, c.ring_pages);
      const size_t piece = std::min<size_t>(c.ring_bytes, 2u << 20);
      std::vector<double> lat;
      const double c0 = thread_cpu_s(), t0 = now_s();
      for (int r = 0; r < c.reads; ++r) {
        const double a = now_s();
        size_t off = 0, roff = 0;
        while (off < c.object_bytes) {
          const size_t k = std::min(piece, c.object_bytes - off);
          if (roff + k > ring.n) roff = 0;
          std::memcpy(ring.p + roff, src.data() + off, k);
          off += k;
          roff += k;
        }
        lat.push_back((now_s() - a) * 1e3);
      }
      const double el = now_s() - t0, cpu = thread_cpu_s() - c0;
      const double gib = static_cast<double>(c.object_bytes) * c.reads / (1 << 30);
      res.gbps = static_cast<double>(c.object_bytes) * c.reads / el / 1e9;
      res.recv_cpu_s_per_gib = cpu / gib;
      res.p50_ms = median(lat);
    } catch (...) {
      err = std::current_exception();
    }
  });
  t.join();
  if (err) std::rethrow_exception(err);
  return res;
}

CeilingResult tcp_ceiling(const CeilingConfig& c) {
  ::signal(SIGPIPE, SIG_IGN);  // a sender outliving a failed receiver must not kill the process
  const size_t obj = c.object_bytes;
  CeilingSource* const ext = c.source;
  Fd mfd(ext ? -1 : memfd_create("ceiling-object", 0));
  if (!ext && mfd.fd < 0) fail("memfd_create");
  if (!ext && ftruncate(mfd.fd, static_cast<off_t>(obj)) != 0) fail("ftruncate");
  const bool thp = !ext && c.zerocopy_send && c.thp_source;
  uint8_t* src = nullptr;  // thp: the object in THP anonymous memory
  if (!ext) {
    // the object's pages on the sender's NUMA node, as the endpoint's source
    // (server/fakegcs.cc): the receiver's copy reads these pages, and pages
    // on the far socket cost it up to 2x per byte (profiles/r2_numa)
    std::exception_ptr fill_err;
    std::thread filler([&] {
      try {
        pin_current_thread(c.send_cpus);
        std::vector<uint8_t> blk(1 << 20);
        for (size_t i = 0; i < blk.size(); ++i) blk[i] = static_cast<uint8_t>(i * 131 + 7);
        if (thp) src = huge_alloc(obj);
        for (size_t off = 0; off < obj; off += blk.size()) {
          const size_t k = std::min(blk.size(), obj - off);
          if (thp) std::memcpy(src + off, blk.data(), k);
          else if (pwrite(mfd.fd, blk.data(), k, static_cast<off_t>(off)) < 0) fail("pwrite");
        }
      } catch (...) {
        fill_err = std::current_exception();
      }
    });
    filler.join();
    if (fill_err) {
      if (src) huge_free(src, obj);
      std::rethrow_exception(fill_err);
    }
  }
  struct SrcFree {
    uint8_t* p;
    size_t n;
    ~SrcFree() {
      if (p) huge_free(p, n);
    }
  } src_free{src, obj};
  Fd ls(socket(AF_INET, SOCK_STREAM, 0));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  set_endpoint_congestion_control(ls.fd);  // on the listener: see Listener (net/socket.cc)
  if (bind(ls.fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || listen(ls.fd, 1) != 0) fail("bind/listen");
  socklen_t al = sizeof(a);
  getsockname(ls.fd, reinterpret_cast<sockaddr*>(&a), &al);

  std::atomic<int> go{0};
  std::atomic<bool> quit{false};
  std::atomic<int> conn_fd{-1};
  std::atomic<int> received{0};  // reads the receiver completed (ext: when end() may run)
  double send_cpu_total = 0;
  std::exception_ptr send_err, recv_err;
  std::thread sender([&] {
    try {
      name_current_thread("ceiling-send");
      pin_current_thread(c.send_cpus);
      Fd s(accept(ls.fd, nullptr, nullptr));
      if (s.fd < 0) fail("accept");
      set_endpoint_congestion_control(s.fd);  // the endpoint's sender, as in server/fakegcs.cc
      int one = 1;
      setsockopt(s.fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      std::vector<uint8_t> copybuf;
      if (!c.zerocopy_send) copybuf.resize(2u << 20);
      Fd sp[2];
      const double c0 = thread_cpu_s();
      double idle_cpu = 0;  // spent spinning for the receiver: not the sender's per-byte cost
      auto wait_for = [&](const std::atomic<int>& a, int past) {
        if (a.load() > past || quit.load()) return;
        const double w0 = thread_cpu_s();
        while (a.load() <= past && !quit.load()) std::this_thread::yield();
        idle_cpu += thread_cpu_s() - w0;
      };
      auto splice_pages = [&](const uint8_t* p, size_t k) {
        if (sp[0].fd < 0) {
          int q[2];
          if (pipe2(q, O_CLOEXEC) != 0) fail("pipe2");
          sp[0].fd = q[0];
          sp[1].fd = q[1];
          (void)fcntl(q[1], F_SETPIPE_SZ, 1 << 20);
        }
        for (size_t done = 0; done < k;) {
          iovec iov{const_cast<uint8_t*>(p + done), k - done};
          const ssize_t v = vmsplice(sp[1].fd, &iov, 1, 0);
          if (v <= 0) fail("vmsplice");
          for (ssize_t left = v; left > 0;) {
            const ssize_t w = splice(sp[0].fd, nullptr, s.fd, nullptr, static_cast<size_t>(left),
                                     SPLICE_F_MOVE | SPLICE_F_MORE);
            if (w <= 0) fail("splice");
            left -= w;
          }
          done += static_cast<size_t>(v);
        }
      };
      for (int r = 0; r < c.reads; ++r) {
        wait_for(go, r);
        if (quit.load()) break;
        if (ext) {
          // one upload's worth: the source stages the object, the pages go
          // out by reference as the transport sends them (grpc_client.cc
          // write_stream), and stay put until the receiver has them all
          ext->begin();
          for (size_t off = 0; off < obj;) {
            auto [p, k] = ext->next(std::min<size_t>(obj - off, 2u << 20));
            if (k == 0) throw std::runtime_error("ceiling: upload source ended early");
            splice_pages(p, k);
            off += k;
          }
          wait_for(received, r);
          ext->end();
          continue;
        }
        off_t off = 0;
        while (static_cast<size_t>(off) < obj) {
          const size_t k = std::min<size_t>(obj - off, 2u << 20);
          if (thp) {
            // vmsplice the pages into a pipe, splice the pipe into the socket
            splice_pages(src + off, k);
            off += static_cast<off_t>(k);
          } else if (c.zerocopy_send) {
            if (sendfile(s.fd, mfd.fd, &off, k) <= 0) fail("sendfile");
          } else {
            if (pread(mfd.fd, copybuf.data(), k, off) != static_cast<ssize_t>(k)) fail("pread");
            size_t done = 0;
            while (done < k) {
              const ssize_t w = send(s.fd, copybuf.data() + done, k - done, MSG_NOSIGNAL);
              if (w <= 0) fail("send");
              done += static_cast<size_t>(w);
            }
            off += static_cast<off_t>(k);
          }
        }
      }
      send_cpu_total = thread_cpu_s() - c0 - idle_cpu;
    } catch (...) {
      send_err = std::current_exception();
      quit.store(true);
      if (int f = conn_fd.load(); f >= 0) ::shutdown(f, SHUT_RDWR);  // unblock the receiver
    }
  });
  CeilingResult res;
  std::thread receiver([&] {
    Fd cs(socket(AF_INET, SOCK_STREAM, 0));
    try {
      name_current_thread("ceiling-recv");
      pin_current_thread(c.recv_cpus);
      if (cs.fd < 0) fail("socket");
      if (c.rcvbuf > 0) setsockopt(cs.fd, SOL_SOCKET, SO_RCVBUF, &c.rcvbuf, sizeof(c.rcvbuf));
      if (connect(cs.fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) fail("connect");
      conn_fd.store(cs.fd);
      Ring ring(c.ring_bytes, c.ring_pages);
      std::vector<double> lat;
      const double c0 = thread_cpu_s(), t0 = now_s();
      for (int r = 0; r < c.reads; ++r) {
        const double st = now_s();
        go.store(r + 1);
        size_t got = 0, roff = 0;
        while (got < obj) {
          if (roff >= ring.n) roff = 0;
          const size_t want = std::min({c.recv_chunk, ring.n - roff, obj - got});
          const ssize_t n = recv(cs.fd, ring.p + roff, want, 0);
          if (n <= 0) {
            if (n == 0) errno = ECONNRESET;
            fail("recv");
          }
          got += static_cast<size_t>(n);
          roff += static_cast<size_t>(n);
        }
        lat.push_back((now_s() - st) * 1e3);
        received.store(r + 1);
      }
      const double el = now_s() - t0, cpu = thread_cpu_s() - c0;
      res.gbps = static_cast<double>(obj) * c.reads / el / 1e9;
      res.recv_cpu_s_per_gib = cpu / (static_cast<double>(obj) * c.reads / (1 << 30));
      res.p50_ms = median(lat);
    } catch (...) {
      recv_err = std::current_exception();
      quit.store(true);
      ::shutdown(ls.fd, SHUT_RDWR);  // a sender still in accept()
    }
    conn_fd.store(-1);
  });
  receiver.join();
  quit.store(true);
  sender.join();
  if (recv_err) std::rethrow_exception(recv_err);
  if (send_err) std::rethrow_exception(send_err);
  res.send_cpu_s_per_gib = send_cpu_total / (static_cast<double>(obj) * c.reads / (1 << 30));
  return res;
}

}  // namespace gcsb
