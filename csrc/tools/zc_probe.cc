// zc_probe: can ONE TCP stream's receive get past the one-core receive copy?
//
// The headline (one gRPC ReadObject stream per read, the reference's
// semantics) is bound by the receiving core's copy_to_user: the kernel copies
// every byte from the socket's pages into the destination on the thread that
// calls recv().  TCP_ZEROCOPY_RECEIVE maps the socket's pages into a VMA of
// the socket instead, so the receiving thread only moves page references and
// the payload copy into the pinned ring can run on several cores at once.
//
// One loopback TCP connection.  A sender thread writes messages of an
// `-hdr`-byte header (send(MSG_MORE), as the endpoint's frame + gRPC prefix)
// followed by `-msg` payload bytes sendfile()d from a memfd at page-aligned
// offsets, so every payload page is a whole-page socket fragment the receiver
// can map.  The receiver:
//   recv        recv() into a 4 x 1 MiB ring (the headline's receive)
//   zc_map      map the payload pages, never touch them (the receive bound)
//   zc_inline   map, then the receiving thread copies the payload to the ring
//   zc_workers  map, and `-workers` threads copy the payload to the ring
// Reports GB/s and the receiving thread's CPU-s/GiB (getrusage per thread).
//
//   zc_probe -mode zc_workers -workers 3 -total 8GiB -send-cpu 2 -recv-cpu 1 -worker-cpus 3,4,5
#include <fcntl.h>
#include <linux/tcp.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <unistd.h>

#include <arpa/inet.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "core/affinity.h"
#include "tools/goflags.h"

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double thread_cpu_s() {
  rusage ru{};
  getrusage(RUSAGE_THREAD, &ru);
  return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}
[[noreturn]] void die(const char* what) { throw std::runtime_error(std::string(what) + ": " + std::strerror(errno)); }

std::vector<int> parse_cpus(const std::string& s) {
  std::vector<int> v;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    if (j > i) v.push_back(std::stoi(s.substr(i, j - i)));
    i = j + 1;
  }
  return v;
}

constexpr size_t kPage = 4096;
constexpr size_t kRegion = 2 << 20;  // VMA reuse granule

struct Job {
  const uint8_t* src;
  uint8_t* dst;
  size_t n;
  uint32_t region;
};

// Single-producer single-consumer job queue; the worker spins while a
// transfer is live (a receive-side poller, not a sleeper).
struct Worker {
  static constexpr size_t kCap = 4096;
  Job q[kCap];
  alignas(64) std::atomic<uint64_t> head{0};
  alignas(64) std::atomic<uint64_t> tail{0};
  alignas(64) std::atomic<bool> stop{false};
  double cpu = 0;
  uint64_t bytes = 0;
};

}  // namespace

int main(int argc, char** argv) {
  gcsb::GoFlags f("zc_probe");
  std::string* mode_p = f.String("mode", "zc_workers", "recv | zc_map | zc_inline | zc_workers");
  std::string* send_cpu_p = f.String("send-cpu", "", "sender CPU list");
  std::string* recv_cpu_p = f.String("recv-cpu", "", "receiving thread CPU list");
  std::string* worker_cpus_p = f.String("worker-cpus", "", "copy worker CPUs, one per worker");
  int64_t* workers_p = f.Int("workers", 3, "copy workers (zc_workers)");
  int64_t* hdr_p = f.Int("hdr", 24, "header bytes before each message's payload");
  int64_t* msg_p = f.Int("msg", 1 << 20, "payload bytes per message");
  int64_t* total_p = f.Int("total", int64_t(8) << 30, "bytes to move");
  int64_t* obj_p = f.Int("object", int64_t(256) << 20, "memfd the payloads are sendfile()d from");
  int64_t* vma_p = f.Int("vma", 64 << 20, "receive VMA bytes (zc modes)");
  int64_t* piece_p = f.Int("piece", 256 << 10, "copy job size (zc_workers)");
  int64_t* lowat_p = f.Int("lowat", 512 << 10, "SO_RCVLOWAT (zc modes)");
  int64_t* copybuf_p = f.Int("copybuf", 4096, "copy buffer for the bytes that cannot be mapped (zc modes)");
  std::string* send_p = f.String("send", "sendfile", "sender: sendfile (page-cache pages) | msg_zerocopy (send(MSG_ZEROCOPY))");
  bool* hint_p = f.Bool("clean-hint", true, "zap a reused region with madvise() first and pass the TLB clean hint");
  f.Parse(argc, argv);
  const std::string mode = *mode_p;
  const size_t H = static_cast<size_t>(*hdr_p), M = static_cast<size_t>(*msg_p);
  const uint64_t total = static_cast<uint64_t>(*total_p), obj = static_cast<uint64_t>(*obj_p);
  const uint64_t nmsg = total / M;
  const size_t VMA = static_cast<size_t>(*vma_p), piece = static_cast<size_t>(*piece_p);
  const bool zc = mode.rfind("zc_", 0) == 0;
  const int nworkers = mode == "zc_workers" ? static_cast<int>(*workers_p) : 0;

  int mfd = memfd_create("zc-probe-object", 0);
  if (mfd < 0 || ftruncate(mfd, static_cast<off_t>(obj)) != 0) die("memfd");
  {
    std::vector<uint8_t> b(1 << 20);
    for (size_t i = 0; i < b.size(); ++i) b[i] = static_cast<uint8_t>(i * 131 + 7);
    for (uint64_t o = 0; o < obj; o += b.size())
      if (pwrite(mfd, b.data(), b.size(), static_cast<off_t>(o)) < 0) die("pwrite");
  }

  int ls = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 || listen(ls, 1) != 0) die("listen");
  socklen_t al = sizeof a;
  getsockname(ls, reinterpret_cast<sockaddr*>(&a), &al);
  int cs = socket(AF_INET, SOCK_STREAM, 0);
  if (connect(cs, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) die("connect");
  int ss = accept(ls, nullptr, nullptr);
  if (ss < 0) die("accept");
  int one = 1;
  setsockopt(cs, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  if (setsockopt(ss, SOL_SOCKET, SO_ZEROCOPY, &one, sizeof one) != 0 && *send_p == "msg_zerocopy") die("SO_ZEROCOPY");
  uint8_t* src = static_cast<uint8_t*>(mmap(nullptr, obj, PROT_READ, MAP_SHARED | MAP_POPULATE, mfd, 0));
  if (src == MAP_FAILED) die("mmap memfd");

  double send_cpu = 0;
  std::thread sender([&] {
    gcsb::pin_current_thread(parse_cpus(*send_cpu_p));
    const double c0 = thread_cpu_s();
    std::vector<uint8_t> hdr(H, 0xA5);
    uint64_t foff = 0;
    for (uint64_t m = 0; m < nmsg; ++m) {
      if (H && send(ss, hdr.data(), H, MSG_MORE | MSG_NOSIGNAL) != static_cast<ssize_t>(H)) die("send hdr");
      if (foff + M > obj) foff = 0;
      if (*send_p == "msg_zerocopy") {
        size_t left = M;
        const uint8_t* p = src + foff;
        while (left) {
          ssize_t w = send(ss, p, left, MSG_ZEROCOPY | MSG_NOSIGNAL);
          if (w <= 0) {
            if (errno == ENOBUFS) {  // drain completions
              char cb[256];
              msghdr mh{};
              mh.msg_control = cb;
              mh.msg_controllen = sizeof cb;
              recvmsg(ss, &mh, MSG_ERRQUEUE);
              continue;
            }
            die("send zerocopy");
          }
          left -= static_cast<size_t>(w), p += w;
        }
        for (;;) {  // completions, non-blocking
          char cb[256];
          msghdr mh{};
          mh.msg_control = cb;
          mh.msg_controllen = sizeof cb;
          if (recvmsg(ss, &mh, MSG_ERRQUEUE | MSG_DONTWAIT) < 0) break;
        }
      } else {
        off_t o = static_cast<off_t>(foff);
        size_t left = M;
        while (left) {
          ssize_t w = sendfile(ss, mfd, &o, left);
          if (w <= 0) die("sendfile");
          left -= static_cast<size_t>(w);
        }
      }
      foff += M;
    }
    send_cpu = thread_cpu_s() - c0;
  });

  const size_t ring_bytes = 4 << 20;
  auto* ring = static_cast<uint8_t*>(mmap(nullptr, ring_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0));
  std::vector<std::unique_ptr<Worker>> ws;
  std::vector<std::thread> wt;
  const size_t nregions = VMA / kRegion;
  std::vector<std::atomic<uint32_t>> pending(nregions);
  for (auto& p : pending) p.store(0);
  const std::vector<int> wcpus = parse_cpus(*worker_cpus_p);
  for (int i = 0; i < nworkers; ++i) {
    ws.emplace_back(new Worker);
    Worker* w = ws.back().get();
    wt.emplace_back([w, i, &wcpus, &pending] {
      if (!wcpus.empty()) gcsb::pin_current_thread({wcpus[static_cast<size_t>(i) % wcpus.size()]});
      const double c0 = thread_cpu_s();
      for (;;) {
        uint64_t t = w->tail.load(std::memory_order_relaxed);
        if (t == w->head.load(std::memory_order_acquire)) {
          if (w->stop.load(std::memory_order_acquire)) break;
          __builtin_ia32_pause();
          continue;
        }
        const Job& j = w->q[t % Worker::kCap];
        std::memcpy(j.dst, j.src, j.n);
        w->bytes += j.n;
        pending[j.region].fetch_sub(1, std::memory_order_release);
        w->tail.store(t + 1, std::memory_order_release);
      }
      w->cpu = thread_cpu_s() - c0;
    });
  }

  double recv_cpu = 0, t0 = 0, t1 = 0;
  uint64_t payload = 0, mapped_bytes = 0, copied_bytes = 0, calls = 0, recv_calls = 0;
  std::thread receiver([&] {
    gcsb::pin_current_thread(parse_cpus(*recv_cpu_p));
    uint8_t* vma = nullptr;
    if (zc) {
      void* m = mmap(nullptr, VMA, PROT_READ, MAP_SHARED, cs, 0);
      if (m == MAP_FAILED) die("mmap socket");
      vma = static_cast<uint8_t*>(m);
      int lw = static_cast<int>(*lowat_p);
      setsockopt(cs, SOL_SOCKET, SO_RCVLOWAT, &lw, sizeof lw);
    }
    std::vector<uint8_t> cbuf(64 << 10);
    // stream parser state: header bytes left, payload bytes left
    size_t hleft = H, pleft = M;
    size_t ring_off = 0;
    uint64_t msgs = 0;
    int rr = 0;
    const uint64_t stream_total = nmsg * (H + M);
    uint64_t got = 0;
    auto consume = [&](const uint8_t* p, size_t n, bool mapped, uint32_t region) {
      while (n) {
        if (hleft) {
          size_t k = std::min(hleft, n);
          hleft -= k, p += k, n -= k;
          continue;
        }
        size_t k = std::min(pleft, n);
        k = std::min(k, ring_bytes - ring_off);
        if (mapped && mode == "zc_workers") {
          for (size_t o = 0; o < k; o += piece) {
            const size_t kk = std::min(piece, k - o);
            Worker* w = ws[static_cast<size_t>(rr++ % nworkers)].get();
            uint64_t h = w->head.load(std::memory_order_relaxed);
            while (h - w->tail.load(std::memory_order_acquire) >= Worker::kCap) __builtin_ia32_pause();
            pending[region].fetch_add(1, std::memory_order_relaxed);
            w->q[h % Worker::kCap] = Job{p + o, ring + ring_off + o, kk, region};
            w->head.store(h + 1, std::memory_order_release);
          }
        } else if (!mapped || mode == "zc_inline") {
          std::memcpy(ring + ring_off, p, k);
        }
        payload += k;
        ring_off = (ring_off + k) % ring_bytes;
        pleft -= k, p += k, n -= k;
        if (!pleft) hleft = H, pleft = M, ++msgs;
      }
    };
    const double c0 = thread_cpu_s();
    t0 = now_s();
    if (!zc) {
      while (got < stream_total) {
        // receive straight into the ring (the headline's copy); headers are
        // parsed out of the ring as they land
        size_t room = ring_bytes - ring_off;
        ssize_t r = recv(cs, ring + ring_off, std::min<uint64_t>(room, stream_total - got), 0);
        if (r <= 0) die("recv");
        ++recv_calls;
        got += static_cast<uint64_t>(r);
        // parse in place: count header/payload split without copying again
        const uint8_t* p = ring + ring_off;
        size_t n = static_cast<size_t>(r);
        while (n) {
          if (hleft) {
            size_t k = std::min(hleft, n);
            hleft -= k, p += k, n -= k;
            continue;
          }
          size_t k = std::min(pleft, n);
          payload += k, pleft -= k, p += k, n -= k;
          if (!pleft) hleft = H, pleft = M, ++msgs;
        }
        copied_bytes += static_cast<uint64_t>(r);
        ring_off = (ring_off + static_cast<size_t>(r)) % ring_bytes;
      }
    } else {
      size_t cursor = 0;
      std::vector<bool> used(nregions, false);
      while (got < stream_total) {
        const uint32_t region = static_cast<uint32_t>(cursor / kRegion);
        const size_t len = (region + 1) * kRegion - cursor;
        bool hint = false;
        if (cursor % kRegion == 0) {
          while (pending[region].load(std::memory_order_acquire)) __builtin_ia32_pause();
          if (used[region] && *hint_p) {
            madvise(vma + cursor, kRegion, MADV_DONTNEED);
          }
          used[region] = true;
          hint = *hint_p;
        } else {
          hint = false;
        }
        if (stream_total - got < static_cast<uint64_t>(*lowat_p)) {
          int lw = static_cast<int>(stream_total - got);
          setsockopt(cs, SOL_SOCKET, SO_RCVLOWAT, &lw, sizeof lw);
        }
        pollfd pf{cs, POLLIN, 0};
        if (getenv("ZC_DEBUG") && calls < 20) std::fprintf(stderr, "poll at cursor %zu\n", cursor);
        if (poll(&pf, 1, -1) < 0) die("poll");
        tcp_zerocopy_receive z{};
        z.address = reinterpret_cast<uint64_t>(vma + cursor);
        z.length = static_cast<uint32_t>(len);
        z.copybuf_address = reinterpret_cast<uint64_t>(cbuf.data());
        z.copybuf_len = static_cast<int32_t>(*copybuf_p);
        if (hint) z.flags = TCP_RECEIVE_ZEROCOPY_FLAG_TLB_CLEAN_HINT;
        socklen_t zl = sizeof z;
        if (getsockopt(cs, IPPROTO_TCP, TCP_ZEROCOPY_RECEIVE, &z, &zl) != 0) die("TCP_ZEROCOPY_RECEIVE");
        ++calls;
        if (getenv("ZC_DEBUG") && calls < 20)
          std::fprintf(stderr, "call %llu cursor %zu len %zu -> mapped %u copybuf %d skip %u inq %u err %d got %llu\n",
                       (unsigned long long)calls, cursor, len, z.length, z.copybuf_len, z.recv_skip_hint, z.inq, z.err,
                       (unsigned long long)got);
        if (z.err) {
          errno = -z.err;
          die("zerocopy err");
        }
        if (z.length) {
          consume(vma + cursor, z.length, true, region);
          mapped_bytes += z.length;
          got += z.length;
          cursor += z.length;
        }
        if (z.copybuf_len > 0) {
          consume(cbuf.data(), static_cast<size_t>(z.copybuf_len), false, region);
          copied_bytes += static_cast<uint64_t>(z.copybuf_len);
          got += static_cast<uint64_t>(z.copybuf_len);
        }
        if (z.recv_skip_hint) {
          size_t want = std::min<size_t>(z.recv_skip_hint, cbuf.size());
          ssize_t r = recv(cs, cbuf.data(), want, 0);
          if (r <= 0) die("recv skip");
          ++recv_calls;
          consume(cbuf.data(), static_cast<size_t>(r), false, region);
          copied_bytes += static_cast<uint64_t>(r);
          got += static_cast<uint64_t>(r);
        }
        // the next mapping starts at a fresh page
        cursor = (cursor + kPage - 1) / kPage * kPage;
        if (cursor >= VMA) cursor = 0;
      }
      for (auto& p : pending)
        while (p.load(std::memory_order_acquire)) __builtin_ia32_pause();
    }
    t1 = now_s();
    recv_cpu = thread_cpu_s() - c0;
    (void)msgs;
  });
  receiver.join();
  sender.join();
  for (auto& w : ws) w->stop.store(true);
  for (auto& t : wt) t.join();
  const double secs = t1 - t0, gib = static_cast<double>(payload) / (1 << 30);
  double wcpu = 0;
  for (auto& w : ws) wcpu += w->cpu;
  std::printf(
      "{\"mode\":\"%s\",\"workers\":%d,\"gbps\":%.2f,\"payload_gib\":%.2f,\"secs\":%.3f,"
      "\"recv_cpu_s_per_gib\":%.4f,\"send_cpu_s_per_gib\":%.4f,\"worker_cpu_s_per_gib\":%.4f,"
      "\"mapped_frac\":%.4f,\"zc_calls\":%llu,\"recv_calls\":%llu}\n",
      mode.c_str(), nworkers, static_cast<double>(payload) / secs / 1e9, gib, secs, recv_cpu / gib, send_cpu / gib,
      wcpu / gib, static_cast<double>(mapped_bytes) / static_cast<double>(mapped_bytes + copied_bytes),
      static_cast<unsigned long long>(calls), static_cast<unsigned long long>(recv_calls));
  return 0;
}
