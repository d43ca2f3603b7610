// O_DIRECT line reader proof of concept (reference small_poc/main.go:1-39).
// The reference hard-codes its path; here it is --path (same default) or the
// first positional argument.  Each line is printed with Go's Println
// semantics (the line keeps its '\n', so an extra newline follows).
#include <string>

#include "tools/fsutil.h"
#include "tools/goflags.h"

using namespace gcsb;

int main(int argc, char** argv) {
  GoFlags f("small_poc");
  auto path = f.String("path", "/usr/local/google/home/princer/gcs/a/b/c/d/e.txt", "File to read line by line");
  auto direct = f.Bool("direct", true, "Open with O_DIRECT");
  f.Parse(argc, argv);
  std::string p = f.Args().empty() ? *path : f.Args()[0];
  std::string err;
  int fd = open_maybe_direct(p, O_RDWR, 0644, *direct, true, &err);
  if (fd < 0) {
    std::printf("%s\n", err.c_str());
    return 0;
  }
  const size_t bs = 1 << 20;
  auto* buf = static_cast<char*>(aligned_buffer(bs));
  std::string pending;
  off_t off = 0;
  for (;;) {
    ssize_t n = ::pread(fd, buf, bs, off);
    if (n < 0) {
      std::printf("%s\n", std::strerror(errno));
      break;
    }
    if (n == 0) break;
    off += n;
    pending.append(buf, static_cast<size_t>(n));
    size_t pos;
    while ((pos = pending.find('\n')) != std::string::npos) {
      std::printf("%s\n", pending.substr(0, pos + 1).c_str());
      pending.erase(0, pos + 1);
    }
  }
  // bufio.ReadString returns the unterminated tail with io.EOF, which the
  // reference drops (it breaks on EOF before printing)
  std::free(buf);
  ::close(fd);
  return 0;
}
