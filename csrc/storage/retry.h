// Retry policy with exponential backoff and full jitter.
//
// Reference: client.SetRetry(WithBackoff(gax.Backoff{Max: 30s, Multiplier: 2}),
// WithPolicy(RetryAlways)) (reference main.go:40-42,179-184).  gax defaults the
// initial pause to 1 s and draws each pause uniformly from (0, cur]; the storage
// library reopens an interrupted read at the byte offset already delivered.
#pragma once
#include <cstdint>
#include <random>
#include <string>

namespace gcsb {

enum class RetryMode { kAlways, kIdempotent, kNever };

struct RetryPolicy {
  RetryMode mode = RetryMode::kAlways;
  double initial_s = 1.0;
  double max_s = 30.0;
  double multiplier = 2.0;
  double max_total_s = 0.0;  // 0 = no deadline (reference uses context.Background)
  int max_attempts = 0;      // 0 = unlimited
};

class Backoff {
 public:
  explicit Backoff(const RetryPolicy& p, uint64_t seed = 0)
      : p_(p), cur_(p.initial_s), rng_(seed ? seed : std::random_device{}()) {}
  // Next pause in seconds (0, cur], then grows cur geometrically up to max.
  double pause() {
    std::uniform_real_distribution<double> u(0.0, 1.0);
    double d = cur_ * (1.0 - u(rng_));  // (0, cur]
    if (d < 1e-9) d = 1e-9;
    cur_ *= p_.multiplier;
    if (cur_ > p_.max_s) cur_ = p_.max_s;
    return d;
  }
  double current() const { return cur_; }

 private:
  RetryPolicy p_;
  double cur_;
  std::mt19937_64 rng_;
};

// Sleep helper that returns early if *cancel becomes true.
void sleep_seconds(double s, const volatile bool* cancel = nullptr);

}  // namespace gcsb
