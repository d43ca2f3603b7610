// Open-handle pressure benchmark (reference benchmark-script/open_file/main.go:1-76).
//
// --dir, --open-files=1: opens <dir>/list_file_<i> O_RDONLY|O_DIRECT for every
// i, prints "All the files are opened now", holds them (--hold-seconds,
// reference 3 min), then closes them.
#include <vector>

#include "core/util.h"
#include "tools/fsutil.h"
#include "tools/goflags.h"

using namespace gcsb;

int main(int argc, char** argv) {
  GoFlags f("open_file");
  auto dir = f.String("dir", "", "Directory file to be opened.");
  auto nfiles = f.Int("open-files", 1, "Number of files to open");
  auto hold_s = f.Float("hold-seconds", 180, "How long to keep the files open");
  auto direct = f.Bool("direct", true, "Open files with O_DIRECT");
  auto fallback = f.Bool("direct-fallback", true, "Fall back to buffered I/O if O_DIRECT is unsupported");
  f.Parse(argc, argv);
  if (dir->empty()) {
    std::fprintf(stderr, "you must set --dir flag\n");
    return 1;
  }
  if (*nfiles <= 0) {
    std::fprintf(stderr, "count not valid\n");
    return 1;
  }
  std::vector<int> fds;
  fds.reserve(static_cast<size_t>(*nfiles));
  int64_t t0 = now_ns();
  for (int64_t i = 0; i < *nfiles; ++i) {
    std::string err;
    int fd = open_maybe_direct(path_join(*dir, "list_file_" + std::to_string(i)), O_RDONLY, 0600, *direct, *fallback,
                               &err);
    if (fd < 0) {
      std::fprintf(stderr, "while opening file: %s\n", err.c_str());
      for (int x : fds) ::close(x);
      return 1;
    }
    fds.push_back(fd);
  }
  std::printf("All the files are opened now\n");
  std::fprintf(stderr, "opened %zu files in %.3f ms\n", fds.size(), (now_ns() - t0) / 1e6);
  std::printf("Waiting for %g seconds\n", *hold_s);
  std::fflush(stdout);
  hold(*hold_s);
  for (int fd : fds)
    if (::close(fd) != 0) {
      std::fprintf(stderr, "while closing the fileHandle: %s\n", std::strerror(errno));
      return 1;
    }
  return 0;
}
