// Directory listing benchmark (reference benchmark-script/list_operation/main.go:1-78).
//
// --dir (required).  Default --mode=ls runs `ls -lah <dir>` like the
// reference's active path (runListingCommandLine, :41-66): prints
// "Listing completed...", pauses (--hold-seconds, reference 3 min), then the
// listing.  --mode=native is the reference's unused Go variant
// (runListingGoScript, :14-36): readdir + stat, one "name size" line per entry.
#include <dirent.h>
#include <sys/stat.h>
#include <sys/wait.h>

#include <algorithm>
#include <vector>

#include "core/util.h"
#include "tools/fsutil.h"
#include "tools/goflags.h"

using namespace gcsb;

int main(int argc, char** argv) {
  GoFlags f("list_operation");
  auto dir = f.String("dir", "", "Directory within which listing performed.");
  auto mode = f.String("mode", "ls", "ls (exec ls -lah) | native (readdir + stat)");
  auto hold_s = f.Float("hold-seconds", 180, "Pause between listing and printing");
  f.Parse(argc, argv);
  if (dir->empty()) {
    std::fprintf(stderr, "you must set --dir flag\n");
    return 1;
  }
  if (*mode == "native") {
    DIR* d = opendir(dir->c_str());
    if (!d) {
      std::fprintf(stderr, "error while readir call: %s\n", std::strerror(errno));
      return 1;
    }
    std::vector<std::string> names;
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n != "." && n != "..") names.push_back(n);
    }
    closedir(d);
    std::sort(names.begin(), names.end());  // os.ReadDir returns sorted entries
    int64_t t0 = now_ns();
    for (const auto& n : names) {
      struct stat st {};
      if (lstat(path_join(*dir, n).c_str(), &st) != 0) {
        std::fprintf(stderr, "while fetching fileInfo: %s\n", std::strerror(errno));
        return 1;
      }
      std::printf("%s %lld\n", n.c_str(), static_cast<long long>(st.st_size));
    }
    std::fprintf(stderr, "listed %zu entries in %.3f ms\n", names.size(), (now_ns() - t0) / 1e6);
    return 0;
  }
  int pipefd[2];
  if (pipe(pipefd) != 0) return 1;
  pid_t pid = fork();
  if (pid == 0) {
    dup2(pipefd[1], 1);
    close(pipefd[0]);
    close(pipefd[1]);
    execlp("ls", "ls", "-lah", dir->c_str(), static_cast<char*>(nullptr));
    _exit(127);
  }
  close(pipefd[1]);
  std::string out;
  char buf[65536];
  ssize_t n;
  while ((n = read(pipefd[0], buf, sizeof(buf))) > 0) out.append(buf, static_cast<size_t>(n));
  close(pipefd[0]);
  int status = 0;
  waitpid(pid, &status, 0);
  if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) {
    std::fprintf(stderr, "error while executing list command\n");
    return 1;
  }
  std::printf("Listing completed...\n");
  std::printf("Waiting for %g seconds\n", *hold_s);
  std::fflush(stdout);
  hold(*hold_s);
  std::printf("%s\n", out.c_str());
  return 0;
}
