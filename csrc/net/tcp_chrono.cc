// TCP_INFO's send chronographs need the kernel's struct tcp_info (glibc's
// <netinet/tcp.h> copy predates them), so this lives apart from socket.cc.
#include <linux/tcp.h>
#include <netinet/in.h>
#include <sys/socket.h>

#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <string>

#include "net/socket.h"

namespace gcsb {

bool read_tcp_chrono(int fd, TcpChrono* out) {
  struct tcp_info ti;
  std::memset(&ti, 0, sizeof(ti));
  socklen_t len = sizeof(ti);
  if (::getsockopt(fd, IPPROTO_TCP, TCP_INFO, &ti, &len) != 0) return false;
  if (len < offsetof(struct tcp_info, tcpi_sndbuf_limited) + sizeof(ti.tcpi_sndbuf_limited)) return false;
  out->busy_us = ti.tcpi_busy_time;
  out->rwnd_limited_us = ti.tcpi_rwnd_limited;
  out->sndbuf_limited_us = ti.tcpi_sndbuf_limited;
  out->cwnd_bytes = static_cast<uint64_t>(ti.tcpi_snd_cwnd) * ti.tcpi_snd_mss;
  return true;
}

const std::string& endpoint_congestion_control() {
  static const std::string cc = [] {
    const char* e = std::getenv("GCSB_SRV_CC");
    std::string v = e && *e ? e : "cubic";
    return v == "default" ? std::string() : v;
  }();
  return cc;
}

void set_loopback_rto_min(int fd) {
  // TCP_RTO_MIN_US (Linux 6.15+; this image's headers predate it): the
  // kernel clamps to its floor (8 ms at HZ 250) and an older kernel refuses
  // the option, harmlessly.
  constexpr int kTcpRtoMinUs = 45;
  const int us = kLoopbackRtoMinUs;
  (void)::setsockopt(fd, IPPROTO_TCP, kTcpRtoMinUs, &us, sizeof(us));
}

void set_endpoint_congestion_control(int fd) {
  const std::string& cc = endpoint_congestion_control();
  if (!cc.empty())
    (void)::setsockopt(fd, IPPROTO_TCP, TCP_CONGESTION, cc.data(), static_cast<socklen_t>(cc.size()));
  set_loopback_rto_min(fd);
}

}  // namespace gcsb
