// Block-read latency benchmark with percentiles (reference
// benchmark-script/ssd_test/main.go:1-189).
//
// Flags: --dir, --threads=1, --block-size=1024 (KB), --file-size=5242880 (KB),
// --read-type=seq (anything else = random), --read-count=1.  Files are
// <dir>/Workload.<i>/0, opened O_DIRECT and size-checked.  One block-offset
// permutation is shared by all threads (reference :112-128).  Each ReadAt is
// timed in microseconds; output is Average/P20/P50/P90/p99/Min/Max in ms with
// floor-index percentiles sorted[size*k/100] (reference :144-164).  Fixed
// (SURVEY.md Q14/Q15/Q16): per-thread latency vectors (the reference appends to
// a shared slice from every goroutine), the corrected divisibility message,
// and errors on stderr.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <random>
#include <sys/stat.h>
#include <thread>
#include <vector>

#include "core/util.h"
#include "tools/fsutil.h"
#include "tools/goflags.h"

using namespace gcsb;

int main(int argc, char** argv) {
  GoFlags f("ssd_test");
  auto dir = f.String("dir", "", "Directory file to be opened.");
  auto threads = f.Int("threads", 1, "Number of threads to read parallel");
  auto block_kb = f.Int("block-size", 1024, "Block size in KB");
  auto file_kb = f.Int("file-size", 5242880, "File size in KB");
  auto read_type = f.String("read-type", "seq", "Read access pattern");
  auto reads = f.Int("read-count", 1, "number of read iteration");
  auto seed = f.Int("seed", 0, "Random permutation seed (0 = time based)");
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
    std::string p = path_join(*dir, "Workload." + std::to_string(i) + "/0");
    fds[i] = open_maybe_direct(p, O_RDONLY, 0600, *direct, *fallback, &err);
    if (fds[i] < 0) {
      std::fprintf(stderr, "while opening file: %s\n", err.c_str());
      return 1;
    }
    struct stat st {};
    if (fstat(fds[i], &st) != 0) {
      std::fprintf(stderr, "while opening file: bad fileHandle\n");
      return 1;
    }
    if (st.st_size != *file_kb * 1024) {
      std::fprintf(stderr, "while opening file: file present is not equal to given file-size\n");
      return 1;
    }
  }
  if (*block_kb <= 0 || *file_kb % *block_kb != 0) {
    std::fprintf(stderr, "file-size should be a multiple of block-size\n");
    return 1;
  }
  const int64_t nblocks = *file_kb / *block_kb;
  std::vector<int64_t> offsets(nblocks);
  for (int64_t i = 0; i < nblocks; ++i) offsets[i] = i;
  if (*read_type != "seq") {
    std::mt19937_64 rng(*seed ? static_cast<uint64_t>(*seed) : static_cast<uint64_t>(now_ns()));
    for (int64_t i = 0; i < nblocks; ++i) {  // Fisher-Yates as in the reference
      std::uniform_int_distribution<int64_t> d(0, i);
      std::swap(offsets[i], offsets[d(rng)]);
    }
  }
  const size_t bs = static_cast<size_t>(*block_kb) * 1024;
  std::vector<std::vector<int64_t>> per_thread(*threads);
  std::atomic<bool> failed{false};
  std::vector<std::thread> th;
  for (int t = 0; t < *threads; ++t)
    th.emplace_back([&, t] {
      auto* buf = static_cast<uint8_t*>(aligned_buffer(bs));
      auto& lat = per_thread[t];
      lat.reserve(static_cast<size_t>(nblocks * *reads));
      for (int64_t r = 0; r < *reads && !failed; ++r)
        for (int64_t b : offsets) {
          int64_t t0 = now_ns();
          ssize_t n = ::pread(fds[t], buf, bs, static_cast<off_t>(b) * static_cast<off_t>(bs));
          int64_t us = (now_ns() - t0) / 1000;
          lat.push_back(us);
          if (n != static_cast<ssize_t>(bs)) {
            failed = true;
            break;
          }
        }
      std::free(buf);
    });
  for (auto& x : th) x.join();
  for (int fd : fds) ::close(fd);
  if (failed) {
    std::fprintf(stderr, "while reading file: error while reading\n");
    return 1;
  }
  std::vector<int64_t> all;
  for (auto& v : per_thread) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  std::printf("read benchmark completed successfully!\n");
  if (all.empty()) return 0;
  int64_t sum = 0;
  for (int64_t v : all) sum += v;
  const size_t size = all.size();
  auto ms = [](int64_t us) { return 0.001 * static_cast<double>(us); };
  std::printf("Average: %.3f ms\n", ms(sum / static_cast<int64_t>(size)));
  std::printf("P20: %.3f ms\n", ms(all[size / 5]));
  std::printf("P50: %.3f ms\n", ms(all[size / 2]));
  std::printf("P90: %.3f ms\n", ms(all[(9 * size) / 10]));
  std::printf("p99: %.3f ms\n", ms(all[(99 * size) / 100]));
  std::printf("Min: %.3f ms\n", ms(all[0]));
  std::printf("Max: %.3f ms\n", ms(all[size - 1]));
  return 0;
}
