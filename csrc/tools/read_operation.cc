// Sequential whole-file read benchmark (reference
// benchmark-script/read_operation/main.go:1-119).
//
// Flags keep the reference's names and defaults: --dir, --threads=1,
// --block-size=256 (KB), --read-count=1.  Files are <dir>/file_<i>, one per
// thread, opened O_RDONLY|O_DIRECT.  Documented deviation: the
// reference's read-count > 1 re-reads nothing (no seek back) and ignores
// --block-size; here every pass preads the whole file from offset 0 in
// --block-size requests, which is what the driver script's matrix intends.
// Added: --hold-seconds (reference: fixed 10 s pause for external memory
// observation), --direct/--direct-fallback.
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "core/util.h"
#include "tools/fsutil.h"
#include "tools/goflags.h"

using namespace gcsb;

int main(int argc, char** argv) {
  GoFlags f("read_operation");
  auto dir = f.String("dir", "", "Directory file to be opened.");
  auto threads = f.Int("threads", 1, "Number of threads to read parallel");
  auto block_kb = f.Int("block-size", 256, "Block size in KB");
  auto reads = f.Int("read-count", 1, "number of read iteration");
  auto hold_s = f.Float("hold-seconds", 10, "Pause after a successful run (external memory observation)");
  auto direct = f.Bool("direct", true, "Open files with O_DIRECT");
  auto fallback = f.Bool("direct-fallback", true, "Fall back to buffered I/O if O_DIRECT is unsupported");
  f.Parse(argc, argv);
  if (dir->empty()) {
    std::fprintf(stderr, "you must set --dir flag\n");
    return 1;
  }
  if (*threads <= 0) {
    std::fprintf(stderr, "threads count not valid\n");
    return 1;
  }
  std::vector<int> fds(*threads, -1);
  for (int i = 0; i < *threads; ++i) {
    std::string err;
    fds[i] = open_maybe_direct(path_join(*dir, "file_" + std::to_string(i)), O_RDONLY, 0600, *direct, *fallback, &err);
    if (fds[i] < 0) {
      std::fprintf(stderr, "while opening file: %s\n", err.c_str());
      return 1;
    }
  }
  const size_t bs = static_cast<size_t>(*block_kb) * 1024;
  std::atomic<uint64_t> total{0};
  std::atomic<bool> failed{false};
  std::string first_err;
  std::mutex mu;
  int64_t t0 = now_ns();
  std::vector<std::thread> th;
  for (int i = 0; i < *threads; ++i)
    th.emplace_back([&, i] {
      auto* buf = static_cast<uint8_t*>(aligned_buffer(bs));
      for (int64_t r = 0; r < *reads && !failed; ++r) {
        off_t off = 0;
        for (;;) {
          ssize_t n = ::pread(fds[i], buf, bs, off);
          if (n < 0) {
            std::lock_guard<std::mutex> lk(mu);
            if (!failed.exchange(true))
              first_err = std::string("while reading and discarding content: ") + std::strerror(errno);
            break;
          }
          if (n == 0) break;
          off += n;
          total += static_cast<uint64_t>(n);
        }
      }
      std::free(buf);
    });
  for (auto& t : th) t.join();
  double dt = (now_ns() - t0) / 1e9;
  if (failed) {
    std::fprintf(stderr, "while reading file: %s\n", first_err.c_str());
  } else {
    std::printf("read benchmark completed successfully!\n");
    std::fprintf(stderr, "read %llu bytes in %.3f s (%.1f MiB/s)\n", static_cast<unsigned long long>(total.load()), dt,
                 dt > 0 ? total.load() / 1048576.0 / dt : 0.0);
    std::printf("Waiting for %g seconds\n", *hold_s);
    std::fflush(stdout);
    hold(*hold_s);
  }
  for (int fd : fds) ::close(fd);
  return failed ? 1 : 0;
}
