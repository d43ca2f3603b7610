// TCP_INFO's send chronographs need the kernel's struct tcp_info (glibc's
// <netinet/tcp.h> copy predates them), so this lives apart from socket.cc.
#include <linux/tcp.h>
#include <arpa/inet.h>
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

// The socket's local address is a loopback one (127/8 or ::1; unbound or
// wildcard listeners are not): only then is a sub-200 ms RTO floor safe.
static bool bound_to_loopback(int fd) {
  sockaddr_storage ss;
  std::memset(&ss, 0, sizeof(ss));
  socklen_t len = sizeof(ss);
  if (::getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &len) != 0) return false;
  if (ss.ss_family == AF_INET) {
    const auto* a = reinterpret_cast<const sockaddr_in*>(&ss);
    return (ntohl(a->sin_addr.s_addr) >> 24) == 127;
  }
  if (ss.ss_family == AF_INET6) {
    const auto* a = reinterpret_cast<const sockaddr_in6*>(&ss);
    return IN6_IS_ADDR_LOOPBACK(&a->sin6_addr);
  }
  return false;
}

void set_endpoint_congestion_control(int fd) {
  const std::string& cc = endpoint_congestion_control();
  if (!cc.empty())
    (void)::setsockopt(fd, IPPROTO_TCP, TCP_CONGESTION, cc.data(), static_cast<socklen_t>(cc.size()));
  // the short RTO floor is for the loopback endpoint only: an endpoint bound
  // to a routable interface for remote clients keeps the kernel's
  if (bound_to_loopback(fd)) set_loopback_rto_min(fd);
}

}  // namespace gcsb
