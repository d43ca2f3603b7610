// splice_probe: what a multiplexed connection's reader thread costs per byte
// when it recv()s every payload into its destination (one core copies all
// streams' bytes), against splice()ing the payload by page reference into a
// per-stream pipe whose owner thread read()s it out (the copy moves to the
// stream's own thread; the reader only moves page references).
//
// One loopback TCP connection.  A sender thread writes messages of a small
// header (frame + gRPC-like prefix) followed by `-msg` bytes sendfile()d from a
// page-cache memfd -- the endpoint's shape (csrc/server/server_grpc.cc).  The
// receiving reader parses the headers through a 16 KiB buffer and hands message
// i's payload to stream i % streams.
//
//   splice_probe -mode recv|splice -streams 8 -msg 1MiB -total 4GiB
//                -send-cpu 2 -recv-cpu 1 -worker-cpus 3,4,5
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <arpa/inet.h>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
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
[[noreturn]] void die(const char* what) {
  throw std::runtime_error(std::string(what) + ": " + std::strerror(errno));
}

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

uint8_t* thp_buf(size_t n) {
  void* m = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) die("mmap");
  madvise(m, n, MADV_HUGEPAGE);
  std::memset(m, 0, n);
  return static_cast<uint8_t*>(m);
}

// One stream's owner: reads its messages' payloads out of its pipe.
struct Stream {
  int pr = -1, pw = -1;
  uint8_t* dst = nullptr;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<size_t> todo;  // byte counts queued in the pipe, in order
  bool done = false;
  double cpu = 0;
  uint64_t bytes = 0;
};

}  // namespace

int main(int argc, char** argv) {
  gcsb::GoFlags f("splice_probe");
  std::string* mode_p = f.String("mode", "splice", "recv | splice");
  std::string* send_cpu_p = f.String("send-cpu", "", "sender CPU list");
  std::string* recv_cpu_p = f.String("recv-cpu", "", "reader CPU list");
  std::string* worker_cpus_p = f.String("worker-cpus", "", "stream owner CPU list (splice mode)");
  int64_t* streams_p = f.Int("streams", 8, "streams (destinations) on the connection");
  int64_t* msg_p = f.Int("msg", 1 << 20, "payload bytes per message");
  int64_t* total_p = f.Int("total", int64_t(4) << 30, "bytes to move");
  int64_t* pipe_p = f.Int("pipe", 1 << 20, "pipe size (F_SETPIPE_SZ)");
  int64_t* obj_p = f.Int("object", int64_t(256) << 20, "memfd object size the payloads are sendfile()d from");
  std::string* src_p = f.String("src", "memfd", "payload source: memfd (sendfile, page cache as written), "
                                "memfd_thp (sendfile, memfd filled through a MADV_HUGEPAGE mapping), "
                                "anon_thp (vmsplice + splice from anonymous THP memory)");
  f.Parse(argc, argv);
  const std::string mode = *mode_p, send_cpu = *send_cpu_p, recv_cpu = *recv_cpu_p, worker_cpus = *worker_cpus_p;
  const int64_t streams = *streams_p, msg = *msg_p, total = *total_p, pipe_sz = *pipe_p, obj = *obj_p;
  const std::string src_kind = *src_p;
  const bool splice_mode = mode == "splice";
  const size_t M = static_cast<size_t>(msg);
  const int64_t nmsg = total / msg;

  int mfd = memfd_create("probe-object", 0);
  if (mfd < 0 || ftruncate(mfd, obj) != 0) die("memfd");
  uint8_t* anon = nullptr;
  long huge_kib = -1;
  {
    std::thread t([&] {
      gcsb::pin_current_thread(parse_cpus(send_cpu));
      std::vector<uint8_t> b(1 << 20);
      for (size_t i = 0; i < b.size(); ++i) b[i] = static_cast<uint8_t>(i * 131 + 7);
      if (src_kind == "memfd") {
        for (int64_t o = 0; o < obj; o += b.size())
          if (pwrite(mfd, b.data(), b.size(), o) < 0) die("pwrite");
      } else if (src_kind == "memfd_thp") {
        void* m = mmap(nullptr, obj, PROT_READ | PROT_WRITE, MAP_SHARED, mfd, 0);
        if (m == MAP_FAILED) die("mmap memfd");
        madvise(m, obj, MADV_HUGEPAGE);
        for (int64_t o = 0; o < obj; o += b.size()) std::memcpy(static_cast<uint8_t*>(m) + o, b.data(), b.size());
        munmap(m, obj);
      } else {
        void* m = mmap(nullptr, obj + (2 << 20), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) die("mmap anon");
        uint8_t* a = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(m) + (2 << 20) - 1) & ~uintptr_t((2 << 20) - 1));
        madvise(a, obj, MADV_HUGEPAGE);
        for (int64_t o = 0; o < obj; o += b.size()) std::memcpy(a + o, b.data(), b.size());
        anon = a;
      }
    });
    t.join();
  }
  {
    // huge pages behind the source: ShmemHugePages / AnonHugePages in meminfo
    FILE* mi = fopen("/proc/meminfo", "r");
    char line[256];
    while (mi && fgets(line, sizeof(line), mi)) {
      long v;
      if (src_kind != "anon_thp" && sscanf(line, "ShmemHugePages: %ld", &v) == 1) huge_kib = v;
      if (src_kind == "anon_thp" && sscanf(line, "AnonHugePages: %ld", &v) == 1) huge_kib = v;
    }
    if (mi) fclose(mi);
  }
  int ls = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || listen(ls, 1) != 0) die("listen");
  socklen_t al = sizeof(a);
  getsockname(ls, reinterpret_cast<sockaddr*>(&a), &al);

  double send_cpu_s = 0;
  std::thread sender([&] {
    gcsb::pin_current_thread(parse_cpus(send_cpu));
    int s = accept(ls, nullptr, nullptr);
    int one = 1;
    setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    const double c0 = thread_cpu_s();
    off_t src = 0;
    for (int64_t i = 0; i < nmsg; ++i) {
      uint8_t hdr[20];
      std::memset(hdr, 0, sizeof(hdr));
      std::memcpy(hdr, &M, sizeof(uint32_t));
      if (send(s, hdr, sizeof(hdr), MSG_MORE) != sizeof(hdr)) die("send");
      if (src + static_cast<off_t>(M) > obj) src = 0;
      off_t o = src;
      size_t left = M;
      if (anon) {
        // vmsplice the pages into a pipe, splice the pipe into the socket
        static thread_local int sp[2] = {-1, -1};
        if (sp[0] < 0) {
          if (pipe2(sp, O_CLOEXEC) != 0) die("pipe2");
          fcntl(sp[1], F_SETPIPE_SZ, 1 << 20);
        }
        while (left) {
          iovec iov{anon + o, std::min<size_t>(left, 1 << 20)};
          ssize_t k = vmsplice(sp[1], &iov, 1, 0);
          if (k <= 0) die("vmsplice");
          o += k;
          left -= static_cast<size_t>(k);
          while (k > 0) {
            ssize_t w = splice(sp[0], nullptr, s, nullptr, static_cast<size_t>(k), SPLICE_F_MOVE | SPLICE_F_MORE);
            if (w <= 0) die("splice out");
            k -= w;
          }
        }
      }
      while (left) {
        ssize_t w = sendfile(s, mfd, &o, left);
        if (w <= 0) die("sendfile");
        left -= static_cast<size_t>(w);
      }
      src += static_cast<off_t>(M);
    }
    send_cpu_s = thread_cpu_s() - c0;
    shutdown(s, SHUT_WR);
    char c;
    while (recv(s, &c, 1, 0) > 0) {
    }
    close(s);
  });

  int cs = socket(AF_INET, SOCK_STREAM, 0);
  int rb = 64 << 20;
  setsockopt(cs, SOL_SOCKET, SO_RCVBUF, &rb, sizeof(rb));
  if (connect(cs, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) die("connect");

  std::vector<Stream> st(static_cast<size_t>(streams));
  std::vector<std::thread> workers;
  const std::vector<int> wcpus = parse_cpus(worker_cpus);
  int got_pipe = 0;
  for (auto& s : st) {
    s.dst = thp_buf(M);
    if (splice_mode) {
      int p[2];
      if (pipe2(p, O_CLOEXEC) != 0) die("pipe2");
      s.pr = p[0];
      s.pw = p[1];
      got_pipe = fcntl(s.pw, F_SETPIPE_SZ, static_cast<int>(pipe_sz));
      if (got_pipe < 0) got_pipe = fcntl(s.pw, F_GETPIPE_SZ);
    }
  }
  if (splice_mode) {
    for (size_t k = 0; k < st.size(); ++k)
      workers.emplace_back([&, k] {
        Stream& s = st[k];
        if (!wcpus.empty()) gcsb::pin_current_thread({wcpus[k % wcpus.size()]});
        const double c0 = thread_cpu_s();
        size_t off = 0;
        for (;;) {
          size_t n;
          {
            std::unique_lock<std::mutex> lk(s.mu);
            s.cv.wait(lk, [&] { return !s.todo.empty() || s.done; });
            if (s.todo.empty()) break;
            n = s.todo.front();
            s.todo.pop_front();
          }
          while (n) {
            if (off == M) off = 0;
            ssize_t r = read(s.pr, s.dst + off, std::min(n, M - off));
            if (r <= 0) die("pipe read");
            n -= static_cast<size_t>(r);
            off += static_cast<size_t>(r);
            s.bytes += static_cast<uint64_t>(r);
          }
        }
        s.cpu = thread_cpu_s() - c0;
      });
  }

  uint64_t splices = 0, spliced = 0, eagain = 0, buffered_copy = 0, recvs = 0;
  double reader_cpu = 0, el = 0;
  std::thread reader([&] {
    gcsb::pin_current_thread(parse_cpus(recv_cpu));
    std::vector<uint8_t> buf(16384);
    size_t pos = 0, end = 0;
    auto fill_hdr = [&](size_t need) {
      while (end - pos < need) {
        if (pos == end) pos = end = 0;
        if (end == buf.size()) {
          std::memmove(buf.data(), buf.data() + pos, end - pos);
          end -= pos;
          pos = 0;
        }
        ssize_t r = recv(cs, buf.data() + end, buf.size() - end, 0);
        if (r <= 0) die("recv hdr");
        end += static_cast<size_t>(r);
      }
    };
    const double c0 = thread_cpu_s(), t0 = now_s();
    for (int64_t i = 0; i < nmsg; ++i) {
      fill_hdr(20);
      pos += 20;
      Stream& s = st[static_cast<size_t>(i) % st.size()];
      size_t left = M, doff = 0;
      const size_t b = std::min(left, end - pos);
      if (b) {
        if (splice_mode) {
          size_t w = 0;
          while (w < b) {
            ssize_t r = write(s.pw, buf.data() + pos + w, b - w);
            if (r <= 0) die("pipe write");
            w += static_cast<size_t>(r);
          }
          std::lock_guard<std::mutex> lk(s.mu);
          s.todo.push_back(b);
        } else {
          std::memcpy(s.dst, buf.data() + pos, b);
        }
        buffered_copy += b;
        pos += b;
        left -= b;
        doff = b;
        if (splice_mode) s.cv.notify_one();
      }
      while (left) {
        ssize_t r;
        if (splice_mode) {
          r = splice(cs, nullptr, s.pw, nullptr, left, SPLICE_F_MOVE | SPLICE_F_NONBLOCK);
          if (r < 0 && errno == EAGAIN) {
            ++eagain;
            r = splice(cs, nullptr, s.pw, nullptr, left, SPLICE_F_MOVE);
          }
          if (r <= 0) die("splice");
          ++splices;
          spliced += static_cast<uint64_t>(r);
          {
            std::lock_guard<std::mutex> lk(s.mu);
            s.todo.push_back(static_cast<size_t>(r));
          }
          s.cv.notify_one();
        } else {
          r = recv(cs, s.dst + doff, left, 0);
          if (r <= 0) die("recv");
          ++recvs;
          doff += static_cast<size_t>(r);
        }
        left -= static_cast<size_t>(r);
      }
    }
    if (splice_mode)
      for (auto& s : st) {
        std::lock_guard<std::mutex> lk(s.mu);
        s.done = true;
        s.cv.notify_one();
      }
    reader_cpu = thread_cpu_s() - c0;
    el = now_s() - t0;
  });
  reader.join();
  for (auto& w : workers) w.join();
  el = std::max(el, 1e-9);
  shutdown(cs, SHUT_WR);
  sender.join();
  const double gib = static_cast<double>(nmsg) * M / (1 << 30);
  double wcpu = 0;
  for (auto& s : st) wcpu += s.cpu;
  std::printf(
      "{\"mode\":\"%s\",\"streams\":%lld,\"msg\":%lld,\"pipe\":%d,\"gbps\":%.2f,\"reader_cpu_s_per_gib\":%.4f,"
      "\"workers_cpu_s_per_gib\":%.4f,\"sender_cpu_s_per_gib\":%.4f,\"splices\":%llu,\"avg_splice_kib\":%.1f,"
      "\"eagain\":%llu,\"recvs\":%llu,\"buffered_copy_frac\":%.4f,\"src\":\"%s\",\"src_huge_kib\":%ld}\n",
      mode.c_str(), (long long)streams, (long long)msg, got_pipe, static_cast<double>(nmsg) * M / el / 1e9,
      reader_cpu / gib, wcpu / gib, send_cpu_s / gib, (unsigned long long)splices,
      splices ? spliced / 1024.0 / splices : 0.0, (unsigned long long)eagain, (unsigned long long)recvs,
      static_cast<double>(buffered_copy) / (static_cast<double>(nmsg) * M), src_kind.c_str(), huge_kib);
  return 0;
}
