// Shared helpers for the POSIX filesystem microbenchmarks (reference
// benchmark-script/*): O_DIRECT opens with an explicit fallback for
// filesystems that reject it (tmpfs/overlay), aligned buffers, sleeps.
#pragma once
#include <fcntl.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

namespace gcsb {

// Opens with O_DIRECT when `direct`; if the filesystem refuses O_DIRECT
// (EINVAL) and `fallback`, retries without it and notes that on stderr.
inline int open_maybe_direct(const std::string& path, int flags, mode_t mode, bool direct, bool fallback,
                             std::string* err) {
  int fd = ::open(path.c_str(), flags | (direct ? O_DIRECT : 0) | O_CLOEXEC, mode);
  if (fd < 0 && direct && errno == EINVAL && fallback) {
    static bool warned = false;
    if (!warned) {
      std::fprintf(stderr, "note: O_DIRECT not supported on this filesystem; using buffered I/O\n");
      warned = true;
    }
    fd = ::open(path.c_str(), flags | O_CLOEXEC, mode);
  }
  if (fd < 0) *err = "open " + path + ": " + std::strerror(errno);
  return fd;
}

inline void* aligned_buffer(size_t n) {
  void* p = nullptr;
  if (posix_memalign(&p, 4096, n ? (n + 4095) / 4096 * 4096 : 4096) != 0) return nullptr;
  return p;
}

inline void hold(double seconds) {
  if (seconds > 0) std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
}

inline std::string path_join(const std::string& dir, const std::string& name) {
  if (dir.empty()) return name;
  return dir.back() == '/' ? dir + name : dir + "/" + name;
}

}  // namespace gcsb
