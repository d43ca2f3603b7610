#include "http1/http1.h"

#include <cstring>

#include "core/util.h"

namespace gcsb {

const std::string* find_header(const Headers& h, std::string_view name) {
  for (const auto& kv : h)
    if (iequals(kv.first, name)) return &kv.second;
  return nullptr;
}

void set_header(Headers& h, const std::string& name, const std::string& value) {
  for (auto& kv : h)
    if (iequals(kv.first, name)) {
      kv.second = value;
      return;
    }
  h.emplace_back(name, value);
}

Http1Pool::Http1Pool(Endpoint ep, SocketOptions opt, int max_conns_per_host, int max_idle_per_host)
    : ep_(std::move(ep)), opt_(opt), max_conns_(max_conns_per_host), max_idle_(max_idle_per_host) {}

Http1Pool::~Http1Pool() = default;

std::unique_ptr<BufferedConn> Http1Pool::get() {
  std::unique_lock<std::mutex> lk(mu_);
  if (max_conns_ > 0) cv_.wait(lk, [&] { return !idle_.empty() || active_ < max_conns_; });
  ++active_;
  if (!idle_.empty()) {
    auto c = std::move(idle_.front());
    idle_.pop_front();
    return c;
  }
  ++dials_;
  lk.unlock();
  try {
    return std::make_unique<BufferedConn>(Conn::dial(ep_, opt_));
  } catch (...) {
    std::lock_guard<std::mutex> g(mu_);
    --active_;
    cv_.notify_one();
    throw;
  }
}

void Http1Pool::put(std::unique_ptr<BufferedConn> c, bool reusable) {
  std::lock_guard<std::mutex> lk(mu_);
  --active_;
  if (reusable && c && c->is_open() && static_cast<int>(idle_.size()) < max_idle_) idle_.push_back(std::move(c));
  cv_.notify_one();
}

void parse_http_headers(BufferedConn& bc, Headers* out) {
  for (;;) {
    std::string line = bc.read_line();
    if (line.empty()) break;
    size_t c = line.find(':');
    if (c == std::string::npos) continue;
    out->emplace_back(std::string(trim(std::string_view(line).substr(0, c))),
                      std::string(trim(std::string_view(line).substr(c + 1))));
  }
}

Http1Exchange::Http1Exchange(Http1Pool& pool, std::vector<RequestDecorator*> decorators)
    : pool_(pool), decorators_(std::move(decorators)) {}

Http1Exchange::~Http1Exchange() { close(); }

const HttpResponseHead& Http1Exchange::send(const std::string& method, const std::string& target, Headers headers,
                                            const void* body, size_t body_len) {
  return send_stream(method, target, std::move(headers), body_len, [&](Conn& c) {
    if (body_len) c.write_all(body, body_len);
  });
}

const HttpResponseHead& Http1Exchange::send_stream(const std::string& method, const std::string& target,
                                                   Headers headers, uint64_t body_len,
                                                   const std::function<void(Conn&)>& write_body) {
  for (auto* d : decorators_) d->decorate(headers);
  if (!find_header(headers, "Host")) headers.emplace(headers.begin(), "Host", pool_.endpoint().host_header());
  if (body_len || method == "POST" || method == "PUT")
    set_header(headers, "Content-Length", std::to_string(body_len));
  std::string req;
  req.reserve(256);
  req += method;
  req += ' ';
  req += pool_.endpoint().base_path + target;
  req += " HTTP/1.1\r\n";
  for (const auto& kv : headers) {
    req += kv.first;
    req += ": ";
    req += kv.second;
    req += "\r\n";
  }
  req += "\r\n";
  // A pooled keep-alive connection may have been closed by the server while
  // idle; retry once on a fresh connection if the write or head read fails
  // before any response byte.
  for (int attempt = 0; attempt < 2; ++attempt) {
    conn_ = pool_.get();
    try {
      conn_->conn().write_all(req.data(), req.size());
      if (body_len) write_body(conn_->conn());
      std::string status = conn_->read_line();
      // "HTTP/1.1 200 OK"
      head_ = HttpResponseHead();
      size_t sp = status.find(' ');
      if (sp == std::string::npos || !starts_with(status, "HTTP/1."))
        throw StorageError("malformed status line: " + status, true);
      head_.status = std::atoi(status.c_str() + sp + 1);
      size_t sp2 = status.find(' ', sp + 1);
      if (sp2 != std::string::npos) head_.reason = status.substr(sp2 + 1);
      parse_http_headers(*conn_, &head_.headers);
      break;
    } catch (const StorageError&) {
      pool_.put(std::move(conn_), false);
      if (attempt == 1) throw;
    }
  }
  if (const auto* te = head_.get("Transfer-Encoding"); te && to_lower(*te).find("chunked") != std::string::npos)
    head_.chunked = true;
  if (const auto* cl = head_.get("Content-Length"); cl && !head_.chunked) head_.content_length = std::stoll(*cl);
  if (const auto* cn = head_.get("Connection"); cn && iequals(*cn, "close")) head_.keep_alive = false;
  body_done_ = false;
  if (method == "HEAD" || head_.status == 204 || head_.status == 304 || (head_.status >= 100 && head_.status < 200)) {
    body_done_ = true;
  } else if (head_.chunked) {
    chunk_left_ = 0;
  } else if (head_.content_length >= 0) {
    body_left_ = head_.content_length;
    body_done_ = body_left_ == 0;
  } else {
    body_left_ = INT64_MAX;  // read until close
    head_.keep_alive = false;
  }
  return head_;
}

size_t Http1Exchange::read_chunked(void* dst, size_t n) {
  if (chunk_left_ == 0) {
    std::string line = conn_->read_line();
    size_t semi = line.find(';');
    chunk_left_ = std::stoll(line.substr(0, semi), nullptr, 16);
    if (chunk_left_ == 0) {
      // trailers
      for (;;) {
        std::string t = conn_->read_line();
        if (t.empty()) break;
      }
      body_done_ = true;
      return 0;
    }
  }
  size_t want = n < static_cast<size_t>(chunk_left_) ? n : static_cast<size_t>(chunk_left_);
  size_t r = conn_->read_some(dst, want);
  if (r == 0) {
    broken_ = true;
    throw StorageError("unexpected EOF in chunked body", true);
  }
  chunk_left_ -= static_cast<int64_t>(r);
  if (chunk_left_ == 0) {
    std::string crlf = conn_->read_line();
    (void)crlf;
  }
  return r;
}

size_t Http1Exchange::read_body(void* dst, size_t n) {
  if (body_done_ || n == 0) return 0;
  try {
    if (head_.chunked) return read_chunked(dst, n);
    size_t want = static_cast<uint64_t>(body_left_) < n ? static_cast<size_t>(body_left_) : n;
    size_t r = conn_->read_some(dst, want);
    if (r == 0) {
      if (body_left_ == INT64_MAX) {
        body_done_ = true;
        return 0;
      }
      broken_ = true;
      throw StorageError("unexpected EOF in body", true);
    }
    if (body_left_ != INT64_MAX) body_left_ -= static_cast<int64_t>(r);
    if (body_left_ == 0) body_done_ = true;
    return r;
  } catch (const StorageError&) {
    broken_ = true;
    throw;
  }
}

uint64_t Http1Exchange::read_body_to_sink(Sink& sink, size_t max_read) {
  uint64_t total = 0;
  while (!body_done_) {
    size_t want = max_read;
    if (!head_.chunked && body_left_ != INT64_MAX && static_cast<uint64_t>(body_left_) < want)
      want = static_cast<size_t>(body_left_);
    Window w = sink.acquire(want);
    size_t cap = w.cap < want ? w.cap : want;
    size_t r = read_body(w.ptr, cap);
    if (r == 0) break;
    sink.commit(r);
    total += r;
  }
  return total;
}

std::string Http1Exchange::read_body_string(size_t max) {
  std::string s;
  char buf[16384];
  for (;;) {
    size_t r = read_body(buf, sizeof(buf));
    if (r == 0) break;
    s.append(buf, r);
    if (s.size() > max) throw StorageError("response body too large", false);
  }
  return s;
}

void Http1Exchange::discard_body() {
  char buf[16384];
  while (read_body(buf, sizeof(buf)) > 0) {
  }
}

void Http1Exchange::close(bool force_drop) {
  if (!conn_) return;
  bool reusable = !force_drop && !broken_ && body_done_ && head_.keep_alive;
  pool_.put(std::move(conn_), reusable);
}

SimpleResponse http_simple_request(const Endpoint& ep, const std::string& method, const std::string& target,
                                   Headers headers, const std::string& body, const SocketOptions& opt) {
  Http1Pool pool(ep, opt, 1, 0);
  Http1Exchange ex(pool, {});
  const auto& h = ex.send(method, target, std::move(headers), body.data(), body.size());
  SimpleResponse r;
  r.status = h.status;
  r.headers = h.headers;
  r.body = ex.read_body_string();
  ex.close(true);
  return r;
}

}  // namespace gcsb
