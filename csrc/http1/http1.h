// HTTP/1.1 client with a keep-alive connection pool.
//
// Reference: CreateHttpClient builds an http.Transport with MaxConnsPerHost=100,
// MaxIdleConnsPerHost=100 and HTTP/2 disabled (reference main.go:62-73), wraps it
// in an oauth2.Transport (main.go:89-95) and a User-Agent round tripper
// (user_agent_round_tripper.go:22-30, main.go:98-101).  Here the same roles are:
//   Http1Pool            — per-endpoint keep-alive pool with a connection cap;
//   RequestDecorator     — ordered header hooks (auth bearer, user agent);
//   Http1Exchange        — one request/response with streaming body reads.
#pragma once
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "net/buffered.h"
#include "net/socket.h"
#include "storage/sink.h"

namespace gcsb {

using Headers = std::vector<std::pair<std::string, std::string>>;

const std::string* find_header(const Headers& h, std::string_view name);
void set_header(Headers& h, const std::string& name, const std::string& value);

// Decorates every outgoing request (RoundTripper middleware equivalent).
class RequestDecorator {
 public:
  virtual ~RequestDecorator() = default;
  virtual void decorate(Headers& headers) = 0;
};

struct HttpResponseHead {
  int status = 0;
  std::string reason;
  Headers headers;
  int64_t content_length = -1;
  bool chunked = false;
  bool keep_alive = true;
  const std::string* get(std::string_view name) const { return find_header(headers, name); }
};

class Http1Pool {
 public:
  Http1Pool(Endpoint ep, SocketOptions opt, int max_conns_per_host, int max_idle_per_host);
  ~Http1Pool();
  std::unique_ptr<BufferedConn> get();  // blocks while max_conns reached
  void put(std::unique_ptr<BufferedConn> c, bool reusable);
  const Endpoint& endpoint() const { return ep_; }
  uint64_t dials() const { return dials_; }

 private:
  Endpoint ep_;
  SocketOptions opt_;
  int max_conns_;
  int max_idle_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::unique_ptr<BufferedConn>> idle_;
  int active_ = 0;
  uint64_t dials_ = 0;
};

// One request/response exchange on a pooled connection.
class Http1Exchange {
 public:
  Http1Exchange(Http1Pool& pool, std::vector<RequestDecorator*> decorators);
  ~Http1Exchange();
  // Sends the request and parses the response head. `body` may be empty.
  const HttpResponseHead& send(const std::string& method, const std::string& target, Headers headers,
                               const void* body = nullptr, size_t body_len = 0);
  // Streaming request body: `write_body` must write exactly body_len bytes.
  const HttpResponseHead& send_stream(const std::string& method, const std::string& target, Headers headers,
                                      uint64_t body_len, const std::function<void(Conn&)>& write_body);
  // Body streaming (Content-Length or chunked). Returns bytes read; 0 at end.
  size_t read_body(void* dst, size_t n);
  // Streams the remaining body into a sink. Returns bytes delivered.
  uint64_t read_body_to_sink(Sink& sink, size_t max_read);
  std::string read_body_string(size_t max = 64 << 20);
  void discard_body();
  // Release the connection (reusable iff the body was fully consumed).
  void close(bool force_drop = false);
  const HttpResponseHead& head() const { return head_; }
  bool body_done() const { return body_done_; }

 private:
  size_t read_chunked(void* dst, size_t n);
  Http1Pool& pool_;
  std::vector<RequestDecorator*> decorators_;
  std::unique_ptr<BufferedConn> conn_;
  HttpResponseHead head_;
  int64_t body_left_ = 0;     // content-length mode
  int64_t chunk_left_ = 0;    // chunked mode: bytes left in the current chunk
  bool body_done_ = false;
  bool broken_ = false;
};

// Parse a response/request head (used by client and server).
void parse_http_headers(BufferedConn& bc, Headers* out);

// One-shot convenience request (token endpoints, metadata, JSON API calls).
struct SimpleResponse {
  int status = 0;
  Headers headers;
  std::string body;
};
SimpleResponse http_simple_request(const Endpoint& ep, const std::string& method, const std::string& target,
                                   Headers headers, const std::string& body, const SocketOptions& opt = {});

}  // namespace gcsb
