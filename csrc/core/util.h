// Small shared helpers: clocks, strings, base64, URL coding, errors.
#pragma once
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace gcsb {

inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
inline int64_t wall_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

// Error with a retryability classification (mirrors the storage library's
// ShouldRetry split: transport resets, 408/429/5xx, gRPC UNAVAILABLE... are
// retryable; 4xx and checksum failures are not).
class StorageError : public std::runtime_error {
 public:
  StorageError(const std::string& msg, bool retryable, int http_status = 0, int grpc_status = -1)
      : std::runtime_error(msg), retryable_(retryable), http_status_(http_status), grpc_status_(grpc_status) {}
  bool retryable() const { return retryable_; }
  int http_status() const { return http_status_; }
  int grpc_status() const { return grpc_status_; }

 private:
  bool retryable_;
  int http_status_;
  int grpc_status_;
};

std::string base64_encode(const void* data, size_t n);
std::string base64_encode(std::string_view s);
bool base64_decode(std::string_view in, std::string* out);
std::string base64url_encode(std::string_view s);  // no padding (JWT)

std::string url_encode(std::string_view s, bool keep_slash = false);
std::string url_decode(std::string_view s);

std::string to_lower(std::string_view s);
std::string_view trim(std::string_view s);
std::vector<std::string_view> split(std::string_view s, char sep);
bool starts_with(std::string_view s, std::string_view p);
bool iequals(std::string_view a, std::string_view b);

// Parse "key=value&..." query string (values URL-decoded).
std::vector<std::pair<std::string, std::string>> parse_query(std::string_view q);

uint32_t be32(const uint8_t* p);
void put_be32(uint8_t* p, uint32_t v);

std::string md5_digest(const void* data, size_t n);  // 16 raw bytes (OpenSSL)

// Minimal JSON string escaping for hand-built JSON documents.
std::string json_escape(std::string_view s);
// Extract a top-level string/number field from a flat JSON object (no nesting
// needed by the callers: token responses, upload initiation bodies).
bool json_get_string(std::string_view json, std::string_view key, std::string* out);
bool json_get_int(std::string_view json, std::string_view key, int64_t* out);

}  // namespace gcsb
