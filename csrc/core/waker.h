// Completion wake-ups taken off a connection's reader thread.
//
// A multiplexed gRPC connection is bound by its one reader thread
// (profiles/r4_ringgeom, r5_wake).  Every stream end wakes the read's worker,
// which sleeps on a condition variable: a futex system call, plus the IPI to
// the worker's core, on the thread that bounds the connection, once per
// 1 MiB read in the reference's 48-worker experiment.  Halving those wake-ups
// on the deferred-CRC discard path gave +12% (profiles/r5_wake).
//
// A Waker moves them to a notifier thread of its own.  The reader only
// queues the stream (a short mutex and a vector push).  The notifier polls
// the queue every poll_us with a timed sleep; its timer slack is set to 1 us.
// It does the futex wakes on a core of the workers' set, never the reader's.
// After idle_ms without work it blocks, and the next post wakes it: that is
// one futex call per idle period, not per read.  The latency cost is up to
// poll_us per read. With several reads in flight per connection, that stays
// off the reader's critical path.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace gcsb {

class Waker {
 public:
  struct Stats {
    uint64_t posts = 0;         // wake-ups queued by readers
    uint64_t batches = 0;       // notifier passes that found work
    uint64_t polls = 0;         // timed sleeps
    uint64_t sleeper_wakes = 0; // posts that had to wake a blocked notifier (futex on the poster)
  };
  Waker(std::vector<int> cpus, int poll_us, int idle_ms = 100);
  ~Waker();
  Waker(const Waker&) = delete;
  Waker& operator=(const Waker&) = delete;
  // Notify every waiter of cv soon; keep holds the object that owns cv alive
  // until then.  The caller has already made the waiters' predicate true
  // under their mutex.
  void post(std::shared_ptr<void> keep, std::condition_variable* cv);
  Stats stats() const;

 private:
  struct Item {
    std::shared_ptr<void> keep;
    std::condition_variable* cv;
  };
  void loop();
  std::vector<int> cpus_;
  int poll_us_;
  int idle_ms_;
  mutable std::mutex mu_;
  std::condition_variable idle_cv_;
  std::vector<Item> q_;
  std::atomic<uint32_t> pending_{0};
  bool sleeping_ = false;
  bool stop_ = false;
  std::atomic<uint64_t> posts_{0}, batches_{0}, polls_{0}, sleeper_wakes_{0};
  std::thread th_;
};

}  // namespace gcsb
