// Block overwrite benchmark (reference benchmark-script/write_operations/main.go:1-139).
//
// Flags: --dir, --threads=1, --block-size=256 (KB), --file-size=1 (KB),
// --write-count=1.  Each thread opens <dir>/file_<i> with
// O_WRONLY|O_CREAT|O_TRUNC|O_DIRECT and, per write-count, writes
// file-size/block-size blocks of fresh random bytes at block offsets with an
// fsync after every block (reference :46-76).  The reference defaults give
// 1/256 = 0 blocks — kept.  --hold-seconds replaces the fixed
// 3-minute pause before close (reference :113-125).
#include <sys/random.h>

#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "core/util.h"
#include "tools/fsutil.h"
#include "tools/goflags.h"

using namespace gcsb;

int main(int argc, char** argv) {
  GoFlags f("write_operations");
  auto dir = f.String("dir", "", "Directory file to be opened.");
  auto threads = f.Int("threads", 1, "Number of threads to read parallel");
  auto block_kb = f.Int("block-size", 256, "Block size in KB");
  auto file_kb = f.Int("file-size", 1, "in KB");
  auto writes = f.Int("write-count", 1, "number of write iteration");
  auto hold_s = f.Float("hold-seconds", 180, "Pause before closing (external memory observation)");
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
    fds[i] = open_maybe_direct(path_join(*dir, "file_" + std::to_string(i)), O_WRONLY | O_CREAT | O_TRUNC, 0644,
                               *direct, *fallback, &err);
    if (fds[i] < 0) {
      std::fprintf(stderr, "while opening file: %s\n", err.c_str());
      return 1;
    }
  }
  const size_t bs = static_cast<size_t>(*block_kb) * 1024;
  const int64_t nblocks = *block_kb > 0 ? *file_kb / *block_kb : 0;
  std::atomic<bool> failed{false};
  std::string first_err;
  std::mutex mu;
  std::atomic<uint64_t> written{0};
  int64_t t0 = now_ns();
  std::vector<std::thread> th;
  for (int i = 0; i < *threads; ++i)
    th.emplace_back([&, i] {
      auto* buf = static_cast<uint8_t*>(aligned_buffer(bs));
      auto fail = [&](const std::string& m) {
        std::lock_guard<std::mutex> lk(mu);
        if (!failed.exchange(true)) first_err = m;
      };
      for (int64_t c = 0; c < *writes && !failed; ++c)
        for (int64_t b = 0; b < nblocks && !failed; ++b) {
          size_t got = 0;
          while (got < bs) {
            ssize_t r = getrandom(buf + got, bs - got, 0);
            if (r <= 0) break;
            got += static_cast<size_t>(r);
          }
          if (got != bs) {
            fail("while generating random bytes");
            break;
          }
          ssize_t w = ::pwrite(fds[i], buf, bs, static_cast<off_t>(b) * static_cast<off_t>(bs));
          if (w != static_cast<ssize_t>(bs)) {
            fail(std::string("while overwriting the file: ") + std::strerror(errno));
            break;
          }
          if (::fsync(fds[i]) != 0) {
            fail(std::string("while syncing the file: ") + std::strerror(errno));
            break;
          }
          written += bs;
        }
      std::free(buf);
    });
  for (auto& t : th) t.join();
  double dt = (now_ns() - t0) / 1e9;
  if (failed) {
    std::fprintf(stderr, "while writing file: %s\n", first_err.c_str());
  } else {
    std::printf("write benchmark completed successfully!\n");
    std::fprintf(stderr, "wrote %llu bytes in %.3f s\n", static_cast<unsigned long long>(written.load()), dt);
    std::printf("Waiting for %g seconds\n", *hold_s);
    std::fflush(stdout);
    hold(*hold_s);
  }
  for (int fd : fds) ::close(fd);
  return failed ? 1 : 0;
}
