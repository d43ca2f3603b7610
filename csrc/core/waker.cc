#include "core/waker.h"

#include <sys/prctl.h>
#include <time.h>

#include <chrono>

#include "core/affinity.h"

namespace gcsb {

Waker::Waker(std::vector<int> cpus, int poll_us, int idle_ms)
    : cpus_(std::move(cpus)), poll_us_(poll_us > 0 ? poll_us : 20), idle_ms_(idle_ms > 0 ? idle_ms : 100) {
  th_ = std::thread([this] { loop(); });
}

Waker::~Waker() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  idle_cv_.notify_one();
  th_.join();
  // anything posted after the last pass: its waiters still get their wake-up
  for (Item& it : q_) it.cv->notify_all();
}

void Waker::post(std::shared_ptr<void> keep, std::condition_variable* cv) {
  bool wake;
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(Item{std::move(keep), cv});
    pending_.store(static_cast<uint32_t>(q_.size()), std::memory_order_release);
    wake = sleeping_;
  }
  posts_.fetch_add(1, std::memory_order_relaxed);
  if (wake) {
    sleeper_wakes_.fetch_add(1, std::memory_order_relaxed);
    idle_cv_.notify_one();
  }
}

Waker::Stats Waker::stats() const {
  Stats s;
  s.posts = posts_.load(std::memory_order_relaxed);
  s.batches = batches_.load(std::memory_order_relaxed);
  s.polls = polls_.load(std::memory_order_relaxed);
  s.sleeper_wakes = sleeper_wakes_.load(std::memory_order_relaxed);
  return s;
}

void Waker::loop() {
  if (!cpus_.empty()) pin_current_thread(cpus_);
  name_current_thread("gcsb-waker");
  prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // poll_us, not poll_us + the default 50 us slack
  using Clock = std::chrono::steady_clock;
  std::vector<Item> batch;
  auto idle_since = Clock::now();
  const timespec nap{0, static_cast<long>(poll_us_) * 1000};
  for (;;) {
    if (pending_.load(std::memory_order_acquire)) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        batch.swap(q_);
        pending_.store(0, std::memory_order_relaxed);
      }
      for (Item& it : batch) it.cv->notify_all();
      batch.clear();  // drops the keep references after the wake-ups
      batches_.fetch_add(1, std::memory_order_relaxed);
      idle_since = Clock::now();
      continue;
    }
    if (Clock::now() - idle_since > std::chrono::milliseconds(idle_ms_)) {
      std::unique_lock<std::mutex> lk(mu_);
      if (stop_) return;
      sleeping_ = true;
      idle_cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      sleeping_ = false;
      if (stop_ && q_.empty()) return;
      idle_since = Clock::now();
      continue;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stop_) return;
    }
    nanosleep(&nap, nullptr);
    polls_.fetch_add(1, std::memory_order_relaxed);
  }
}

}  // namespace gcsb
