// HTTP/1.1 front end of the synthetic GCS server.
#include <sys/socket.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <set>
#include <thread>

#include "core/content.h"
#include "core/crc32c.h"
#include "core/json.h"
#include "core/util.h"
#include "http1/http1.h"
#include "net/buffered.h"
#include "server/fakegcs.h"
#include "server/media.h"
#include "storage/auth.h"
#include "storage/client.h"

namespace gcsb {
namespace {

struct Request {
  std::string method, target, path, query_str;
  std::vector<std::pair<std::string, std::string>> query;
  Headers headers;
  std::string body;
  // Resumable-upload chunk bodies are not buffered: the handler streams them
  // from the socket (CRC + store while the client is still sending).  Bytes
  // of a deferred body not consumed by the handler are drained after it.
  uint64_t deferred = 0;
  const std::string* header(std::string_view n) const { return find_header(headers, n); }
  std::string q(const std::string& k, const std::string& dflt = "") const {
    for (const auto& kv : query)
      if (kv.first == k) return kv.second;
    return dflt;
  }
  bool has_q(const std::string& k) const {
    for (const auto& kv : query)
      if (kv.first == k) return true;
    return false;
  }
};

struct CloseConnection {};

const char* reason_phrase(int st) {
  switch (st) {
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 206: return "Partial Content";
    case 308: return "Resume Incomplete";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 408: return "Request Timeout";
    case 412: return "Precondition Failed";
    case 416: return "Requested Range Not Satisfiable";
    case 429: return "Too Many Requests";
    case 500: return "Internal Server Error";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
    default: return "Status";
  }
}

void write_head(Conn& c, int status, const Headers& h, uint64_t content_length) {
  std::string s = "HTTP/1.1 " + std::to_string(status) + " " + reason_phrase(status) + "\r\n";
  for (const auto& kv : h) s += kv.first + ": " + kv.second + "\r\n";
  s += "Content-Length: " + std::to_string(content_length) + "\r\n\r\n";
  c.write_all(s.data(), s.size());
}

void respond(Conn& c, int status, Headers h, const std::string& body,
             const std::string& ctype = "application/json; charset=UTF-8") {
  if (!body.empty() || status != 308) h.emplace_back("Content-Type", ctype);
  h.emplace_back("Server", "gcsb-fakegcs");
  write_head(c, status, h, body.size());
  if (!body.empty()) c.write_all(body.data(), body.size());
}

class Http1Handler {
 public:
  Http1Handler(FakeGcsServer& srv, BufferedConn& bc) : srv_(srv), bc_(bc), c_(bc.conn()) {}

  void run() {
    for (;;) {
      Request r;
      // request bodies (upload chunks) land in a buffer reused across the
      // connection's requests: warm pages instead of fresh faults per chunk
      r.body.swap(body_buf_);
      r.body.clear();
      try {
        if (!read_request(&r)) return;
      } catch (const StorageError&) {
        return;
      }
      ++srv_.stats().http_requests;
      bool keep = true;
      if (const auto* cn = r.header("Connection"); cn && iequals(*cn, "close")) keep = false;
      try {
        dispatch(r);
        if (r.deferred) bc_.skip(r.deferred);
      } catch (const CloseConnection&) {
        return;
      } catch (const StorageError&) {
        return;
      } catch (const std::exception& e) {
        try {
          respond(c_, 500, {}, json_error(500, e.what(), "backendError"));
        } catch (...) {
          return;
        }
      }
      if (!keep) return;
      if (r.body.capacity() <= (64u << 20)) body_buf_.swap(r.body);
    }
  }

 private:
  bool read_request(Request* r) {
    std::string line;
    do {
      line = bc_.read_line();  // EOF between requests throws -> orderly close
    } while (line.empty());
    auto parts = split(line, ' ');
    if (parts.size() < 3) throw StorageError("bad request line", false);
    r->method = std::string(parts[0]);
    r->target = std::string(parts[1]);
    size_t qm = r->target.find('?');
    r->path = r->target.substr(0, qm);
    if (qm != std::string::npos) {
      r->query_str = r->target.substr(qm + 1);
      r->query = parse_query(r->query_str);
    }
    parse_http_headers(bc_, &r->headers);
    const auto* te = r->header("Transfer-Encoding");
    if (te && to_lower(*te).find("chunked") != std::string::npos) {
      for (;;) {
        std::string sz = bc_.read_line();
        size_t n = std::stoull(sz, nullptr, 16);
        if (n == 0) {
          while (!bc_.read_line().empty()) {
          }
          break;
        }
        size_t old = r->body.size();
        r->body.resize(old + n);
        bc_.read_exact(&r->body[old], n);
        bc_.read_line();
      }
    } else if (const auto* cl = r->header("Content-Length")) {
      size_t n = std::stoull(*cl);
      if (r->method == "PUT" && starts_with(r->path, "/upload/storage/v1/b/") && r->has_q("upload_id")) {
        r->deferred = n;
        srv_.stats().bytes_received += n;
        return true;
      }
      r->body.resize(n);
      if (n) bc_.read_exact(&r->body[0], n);
    }
    srv_.stats().bytes_received += r->body.size();
    return true;
  }

  bool check_auth(const Request& r) {
    if (!srv_.config().require_auth) return true;
    const auto* a = r.header("Authorization");
    if (a && starts_with(*a, "Bearer ") && srv_.token_valid(a->substr(7))) return true;
    ++srv_.stats().auth_failures;
    respond(c_, 401, {{"WWW-Authenticate", "Bearer realm=\"https://accounts.google.com/\""}},
            json_error(401, "Invalid Credentials", "authError"));
    return false;
  }

  // Returns true if a fault response was sent.
  bool maybe_fail(bool xml) {
    auto& f = srv_.faults();
    int n = f.fail_next.load();
    while (n > 0) {
      if (f.fail_next.compare_exchange_weak(n, n - 1)) {
        ++srv_.stats().faults_injected;
        int st = f.fail_status.load();
        if (xml)
          respond(c_, st, {}, "<?xml version='1.0' encoding='UTF-8'?><Error><Code>ServiceUnavailable</Code></Error>",
                  "application/xml; charset=UTF-8");
        else
          respond(c_, st, {}, json_error(st, "injected fault", "backendError"));
        return true;
      }
    }
    return false;
  }

  void dispatch(Request& r) {
    const std::string& p = r.path;
    if (p == "/token" && r.method == "POST") return token(r);
    if (starts_with(p, "/computeMetadata/v1/instance/service-accounts/default/token")) return metadata_token(r);
    if (p == "/_gcsb/stats") return stats();
    if (p == "/_gcsb/faults" && r.method == "POST") return faults(r);
    if (starts_with(p, "/upload/storage/v1/b/")) {
      if (!check_auth(r)) return;
      return upload(r, p.substr(std::strlen("/upload/storage/v1/b/")));
    }
    std::string rest;
    if (starts_with(p, "/storage/v1/b/")) rest = p.substr(std::strlen("/storage/v1/b/"));
    else if (starts_with(p, "/download/storage/v1/b/")) rest = p.substr(std::strlen("/download/storage/v1/b/"));
    if (!rest.empty()) {
      if (!check_auth(r)) return;
      return json_api(r, rest);
    }
    if (!check_auth(r)) return;
    return xml_api(r);
  }

  void token(const Request& r) {
    auto form = parse_query(r.body);
    std::string grant, assertion;
    for (auto& kv : form) {
      if (kv.first == "grant_type") grant = kv.second;
      if (kv.first == "assertion") assertion = kv.second;
    }
    if (grant == "urn:ietf:params:oauth:grant-type:jwt-bearer") {
      auto parts = split(assertion, '.');
      if (parts.size() != 3) return respond(c_, 400, {}, "{\"error\":\"invalid_grant\"}");
      if (!srv_.config().jwt_public_key_pem.empty()) {
        std::string sig;
        base64_decode(parts[2], &sig);
        std::string signed_part = std::string(parts[0]) + "." + std::string(parts[1]);
        if (!rs256_verify(srv_.config().jwt_public_key_pem, signed_part, sig))
          return respond(c_, 400, {}, "{\"error\":\"invalid_grant\",\"error_description\":\"Invalid JWT Signature.\"}");
      }
      std::string claims;
      base64_decode(parts[1], &claims);
      std::string scope;
      json_get_string(claims, "scope", &scope);
      if (scope.empty()) return respond(c_, 400, {}, "{\"error\":\"invalid_scope\"}");
    } else if (grant != "refresh_token") {
      return respond(c_, 400, {}, "{\"error\":\"unsupported_grant_type\"}");
    }
    respond(c_, 200, {},
            "{\"access_token\":\"" + srv_.issue_token() + "\",\"expires_in\":3599,\"token_type\":\"Bearer\"}");
  }

  void metadata_token(const Request& r) {
    const auto* f = r.header("Metadata-Flavor");
    if (!f || *f != "Google") return respond(c_, 403, {}, "Missing Metadata-Flavor:Google header.", "text/html");
    respond(c_, 200, {{"Metadata-Flavor", "Google"}},
            "{\"access_token\":\"" + srv_.issue_token() + "\",\"expires_in\":3599,\"token_type\":\"Bearer\"}");
  }

  void stats() {
    auto& s = srv_.stats();
    Json j = Json::object();
    j.set("connections", Json::num(static_cast<double>(s.connections.load())));
    j.set("http_requests", Json::num(static_cast<double>(s.http_requests.load())));
    j.set("grpc_calls", Json::num(static_cast<double>(s.grpc_calls.load())));
    j.set("bytes_sent", Json::num(static_cast<double>(s.bytes_sent.load())));
    j.set("bytes_received", Json::num(static_cast<double>(s.bytes_received.load())));
    j.set("faults_injected", Json::num(static_cast<double>(s.faults_injected.load())));
    j.set("auth_failures", Json::num(static_cast<double>(s.auth_failures.load())));
    j.set("objects", Json::num(static_cast<double>(srv_.store().count())));
    respond(c_, 200, {}, j.dump());
  }

  void faults(const Request& r) {
    Json j = Json::parse(r.body);
    auto& f = srv_.faults();
    if (j.get("fail_next")) f.fail_next = static_cast<int>(j.get_int("fail_next"));
    if (j.get("fail_status")) f.fail_status = static_cast<int>(j.get_int("fail_status"));
    if (j.get("disconnect_at")) f.disconnect_at = j.get_int("disconnect_at");
    if (j.get("disconnect_count")) f.disconnect_count = static_cast<int>(j.get_int("disconnect_count"));
    if (j.get("corrupt_at")) f.corrupt_at = j.get_int("corrupt_at");
    if (j.get("corrupt_count")) f.corrupt_count = static_cast<int>(j.get_int("corrupt_count"));
    if (j.get("throttle_bps")) f.throttle_bps = j.get_int("throttle_bps");
    if (j.get("latency_ms")) f.latency_ms = static_cast<int>(j.get_int("latency_ms"));
    if (j.get("stall_at")) f.stall_at = j.get_int("stall_at");
    if (j.get("stall_ms")) f.stall_ms = static_cast<int>(j.get_int("stall_ms"));
    if (j.get("stall_count")) f.stall_count = static_cast<int>(j.get_int("stall_count"));
    respond(c_, 200, {}, "{}");
  }

  void send_media(const Request& r, const StoredObject& o, bool xml) {
    const std::string gen = r.q("generation");
    if (r.has_q("generation") && std::strtoll(gen.c_str(), nullptr, 10) != o.generation)
      return respond(c_, 404, {}, json_error(404, "No such object: " + o.bucket + "/" + o.name + "#" + gen,
                                             "notFound"));
    if (maybe_fail(xml)) return;
    MediaPlan mp = plan_media(o, r.header("Range"), nullptr);
    if (mp.status >= 400) return respond(c_, mp.status, mp.headers, mp.body, mp.content_type);
    auto& f = srv_.faults();
    if (int lat = f.latency_ms.load()) std::this_thread::sleep_for(std::chrono::milliseconds(lat));
    write_head(c_, mp.status, mp.headers, mp.len);
    if (r.method == "HEAD") return;
    stream_bytes(o, mp.start, mp.len);
  }

  void stream_bytes(const StoredObject& o, uint64_t start, uint64_t len) {
    auto& f = srv_.faults();
    int64_t disc = f.disconnect_count.load() > 0 ? f.disconnect_at.load() : -1;
    const int64_t disc_at = disc;
    int64_t corrupt = f.corrupt_count.load() > 0 ? f.corrupt_at.load() : -1;
    int64_t bps = f.throttle_bps.load();
    int64_t stall = f.stall_count.load() > 0 ? f.stall_at.load() : -1;
    int64_t t0 = now_ns();
    uint64_t sent = 0;
    // send chronographs for big bodies only: two TCP_INFO calls per 1 MiB
    // body would cost the many-small-reads blocks a few % of a core
    TcpChrono chrono0;
    const bool chrono_ok = len >= kChronoMinBody && read_tcp_chrono(c_.fd(), &chrono0);
    // bytes per send call (1-16 MiB measured equal, profiles/r3_twins/http_piece)
    constexpr uint64_t piece_max = uint64_t(8) << 20;
    while (sent < len) {
      uint64_t off = start + sent;
      uint64_t n = std::min<uint64_t>(piece_max, len - sent);
      if (bps > 0) n = std::min<uint64_t>(n, std::max<int64_t>(4096, bps / 100));
      if (stall >= 0 && static_cast<int64_t>(off) <= stall && static_cast<int64_t>(off + n) > stall) {
        if (static_cast<int64_t>(off) < stall) {
          n = static_cast<uint64_t>(stall) - off;  // send up to the stall point first
        } else {
          stall = -1;
          if (f.stall_count.fetch_sub(1) > 0) {
            ++srv_.stats().faults_injected;
            std::this_thread::sleep_for(std::chrono::milliseconds(f.stall_ms.load()));
          }
          continue;
        }
      }
      if (disc >= 0 && static_cast<int64_t>(off + n) > disc && static_cast<int64_t>(off) <= disc) {
        disc = -1;  // at most once per response
        // claim one of the remaining faults (concurrent responses race for it)
        if (f.disconnect_count.fetch_sub(1) > 0) {
          uint64_t k = static_cast<uint64_t>(disc_at) - off;
          if (k) c_.write_all(o.bytes(off, k), k);
          ++srv_.stats().faults_injected;
          srv_.stats().bytes_sent += sent + k;
          ::shutdown(c_.fd(), SHUT_RDWR);
          throw CloseConnection{};
        }
        continue;
      }
      if (corrupt >= 0 && static_cast<int64_t>(off) <= corrupt && static_cast<int64_t>(off + n) > corrupt) {
        const uint64_t k = static_cast<uint64_t>(corrupt) - off;
        corrupt = -1;
        if (f.corrupt_count.fetch_sub(1) > 0) {
          ++srv_.stats().faults_injected;
          if (k) c_.write_all(o.bytes(off, k), k);
          uint8_t bad = static_cast<uint8_t>(o.bytes(off + k, 1)[0] ^ 0x5A);
          c_.write_all(&bad, 1);
          sent += k + 1;
        }
        continue;
      }
      int ffd = -1;
      uint64_t foff = 0;
      if (const uint8_t* sp = srv_.config().zero_copy && srv_.config().send_vmsplice ? o.splice_bytes(off, n) : nullptr)
        c_.splice_user_all(sp, n);  // THP pattern pages by reference, no copy
      else if (srv_.config().zero_copy && o.file_range(off, &ffd, &foff))
        c_.sendfile_all(ffd, foff, n);  // page references, no user-space copy
      else
        c_.write_all(o.bytes(off, n), n);
      sent += n;
      if (bps > 0) {
        int64_t due = t0 + static_cast<int64_t>(sent * 1e9 / static_cast<double>(bps));
        int64_t now = now_ns();
        if (due > now) std::this_thread::sleep_for(std::chrono::nanoseconds(due - now));
      }
    }
    srv_.stats().bytes_sent += sent;
    srv_.stats().note_body_send(c_.fd(), chrono0, chrono_ok, t0);
  }

  void xml_api(Request& r) {
    // /<bucket>/<object>
    std::string p = r.path.substr(1);
    size_t sl = p.find('/');
    if (sl == std::string::npos || sl + 1 >= p.size()) {
      return respond(c_, 400, {}, "<Error><Code>InvalidURI</Code></Error>", "application/xml");
    }
    std::string bucket = url_decode(p.substr(0, sl));
    std::string name = url_decode(p.substr(sl + 1));
    if (r.method == "GET" || r.method == "HEAD") {
      auto o = srv_.store().get(bucket, name);
      if (!o)
        return respond(c_, 404, {},
                       "<?xml version='1.0' encoding='UTF-8'?><Error><Code>NoSuchKey</Code><Message>The specified "
                       "key does not exist.</Message></Error>",
                       "application/xml; charset=UTF-8");
      return send_media(r, *o, true);
    }
    if (r.method == "PUT") {
      Blob data;
      data.append(r.body.data(), r.body.size());
      const auto* ct = r.header("Content-Type");
      auto o = srv_.store().put(bucket, name, std::move(data), ct ? *ct : "");
      return respond(c_, 200, {{"ETag", "\"" + std::to_string(o->generation) + "\""},
                               {"x-goog-generation", std::to_string(o->generation)},
                               {"x-goog-hash", "crc32c=" + crc32c_b64(o->crc32c)}},
                     "", "text/html");
    }
    if (r.method == "DELETE") {
      if (!srv_.store().remove(bucket, name))
        return respond(c_, 404, {}, "<Error><Code>NoSuchKey</Code></Error>", "application/xml");
      return respond(c_, 204, {}, "", "text/html");
    }
    respond(c_, 405, {}, "", "text/html");
  }

  void json_api(Request& r, const std::string& rest) {
    size_t sl = rest.find('/');
    std::string bucket = url_decode(rest.substr(0, sl));
    std::string tail = sl == std::string::npos ? "" : rest.substr(sl);
    if (tail == "/o" || tail == "/o/") {
      if (r.method != "GET") return respond(c_, 405, {}, json_error(405, "method not allowed", "invalid"));
      return list(r, bucket);
    }
    if (!starts_with(tail, "/o/")) return respond(c_, 404, {}, json_error(404, "Not Found", "notFound"));
    static const std::string kCompose = "/compose";
    if (r.method == "POST" && tail.size() > 3 + kCompose.size() &&
        tail.compare(tail.size() - kCompose.size(), kCompose.size(), kCompose) == 0) {
      return compose(r, bucket, url_decode(tail.substr(3, tail.size() - 3 - kCompose.size())));
    }
    std::string name = url_decode(tail.substr(3));
    if (r.method == "DELETE") {
      if (!srv_.store().remove(bucket, name))
        return respond(c_, 404, {}, json_error(404, "No such object: " + bucket + "/" + name, "notFound"));
      return respond(c_, 204, {}, "", "text/html");
    }
    auto o = srv_.store().get(bucket, name);
    if (!o) return respond(c_, 404, {}, json_error(404, "No such object: " + bucket + "/" + name, "notFound"));
    if (r.q("alt") == "media") return send_media(r, *o, false);
    respond(c_, 200, {}, object_json(*o).dump());
  }

  // POST /storage/v1/b/<b>/o/<dest>/compose
  //   {"sourceObjects": [{"name": ...}, ...], "destination": {"contentType": ...}}
  void compose(const Request& r, const std::string& bucket, const std::string& dest) {
    Json j;
    try {
      j = Json::parse(r.body);
    } catch (const std::exception&) {
      return respond(c_, 400, {}, json_error(400, "Parse Error", "parseError"));
    }
    std::vector<std::string> names;
    if (const Json* so = j.get("sourceObjects"); so && so->is_array())
      for (const auto& e : so->items())
        if (const Json* n = e.get("name"); n && n->is_string()) names.push_back(n->as_string());
    std::string ct;
    if (const Json* d = j.get("destination"))
      if (const Json* c = d->get("contentType"); c && c->is_string()) ct = c->as_string();
    std::string err;
    auto o = srv_.store().compose(bucket, dest, names, ct, &err);
    if (!o) return respond(c_, err.find("not found") != std::string::npos ? 404 : 400, {}, json_error(400, err, "invalid"));
    respond(c_, 200, {}, object_json(*o, false).dump());
  }

  void list(const Request& r, const std::string& bucket) {
    std::string prefix = r.q("prefix");
    std::string delim = r.q("delimiter");
    size_t max = static_cast<size_t>(std::max(1, std::min(5000, std::atoi(r.q("maxResults", "1000").c_str()))));
    std::string start_after = r.q("pageToken");
    Json items = Json::array();
    Json prefixes = Json::array();
    std::set<std::string> seen_prefixes;
    std::string last;
    size_t emitted = 0;
    bool more = false;
    std::string cursor = start_after;
    while (emitted < max) {
      auto batch = srv_.store().list(bucket, prefix, cursor, max - emitted + 1);
      if (batch.empty()) break;
      for (auto& o : batch) {
        cursor = o->name;
        if (emitted >= max) {
          more = true;
          break;
        }
        if (!delim.empty()) {
          size_t d = o->name.find(delim, prefix.size());
          if (d != std::string::npos) {
            std::string pf = o->name.substr(0, d + delim.size());
            if (seen_prefixes.insert(pf).second) {
              prefixes.push(Json::str(pf));
              ++emitted;
              last = o->name;
            }
            continue;
          }
        }
        items.push(object_json(*o));
        ++emitted;
        last = o->name;
      }
      if (more || batch.size() < max - emitted + 1) break;
    }
    if (!more && emitted >= max) more = !srv_.store().list(bucket, prefix, last, 1).empty();
    Json j = Json::object();
    j.set("kind", Json::str("storage#objects"));
    if (!items.items().empty()) j.set("items", items);
    if (!prefixes.items().empty()) j.set("prefixes", prefixes);
    if (more) j.set("nextPageToken", Json::str(last));
    respond(c_, 200, {}, j.dump());
  }

  void upload(Request& r, const std::string& rest) {
    size_t sl = rest.find('/');
    std::string bucket = url_decode(rest.substr(0, sl));
    std::string type = r.q("uploadType");
    if (r.method == "POST" && type == "media") {
      std::string name = r.q("name");
      if (name.empty()) return respond(c_, 400, {}, json_error(400, "Required parameter: name", "required"));
      Blob data;
      data.append(r.body.data(), r.body.size());
      const uint32_t data_crc = gcsb::crc32c(data.data(), data.size());
      if (const auto* gh = r.header("x-goog-hash")) {
        bool has = false;
        uint32_t crc = 0;
        std::string md5;
        parse_goog_hash(*gh, &has, &crc, &md5);
        if (has && crc != data_crc)
          return respond(c_, 400, {}, json_error(400, "Provided CRC32C doesn't match calculated CRC32C", "invalid"));
      }
      const auto* ct = r.header("Content-Type");
      auto o = srv_.store().put(bucket, name, std::move(data), ct ? *ct : "", &data_crc);
      return respond(c_, 200, {}, object_json(*o, false).dump());
    }
    if (r.method == "POST" && type == "resumable") {
      std::string name = r.q("name");
      std::string ctype = "application/octet-stream";
      bool has_crc = false;
      uint32_t crc = 0;
      if (!r.body.empty()) {
        Json md = Json::parse(r.body);
        if (name.empty()) name = md.get_string("name");
        ctype = md.get_string("contentType", ctype);
        if (const Json* c = md.get("crc32c"); c && c->is_string()) has_crc = crc32c_from_b64(c->as_string(), &crc);
      }
      if (const auto* xct = r.header("X-Upload-Content-Type")) ctype = *xct;
      int64_t expected = -1;
      if (const auto* xl = r.header("X-Upload-Content-Length")) expected = std::stoll(*xl);
      if (name.empty()) return respond(c_, 400, {}, json_error(400, "Required parameter: name", "required"));
      auto s = srv_.store().start_upload(bucket, name, ctype, expected);
      s->has_crc = has_crc;
      s->crc = crc;
      std::string host = "127.0.0.1:" + std::to_string(srv_.port());
      if (const auto* hh = r.header("Host")) host = *hh;
      return respond(c_, 200,
                     {{"Location", "http://" + host + "/upload/storage/v1/b/" + url_encode(bucket) +
                                       "/o?uploadType=resumable&upload_id=" + s->id},
                      {"X-GUploader-UploadID", s->id}},
                     "", "text/plain");
    }
    if (r.method == "PUT" && r.has_q("upload_id")) {
      auto s = srv_.store().find_upload(r.q("upload_id"));
      if (!s) return respond(c_, 404, {}, json_error(404, "No such upload", "notFound"));
      std::lock_guard<std::mutex> lk(s->mu);
      if (s->finalized) return respond(c_, 200, {}, object_json(*s->result, false).dump());
      std::string cr;
      if (const auto* h = r.header("Content-Range")) cr = *h;
      // "bytes a-b/total" | "bytes a-b/*" | "bytes */total" | "bytes */*"
      int64_t a = -1, b = -1, total = -1;
      if (starts_with(cr, "bytes ")) {
        std::string v = cr.substr(6);
        size_t slash = v.find('/');
        std::string range = v.substr(0, slash), tot = slash == std::string::npos ? "*" : v.substr(slash + 1);
        if (tot != "*") total = std::stoll(tot);
        if (range != "*") {
          size_t dash = range.find('-');
          a = std::stoll(range.substr(0, dash));
          b = std::stoll(range.substr(dash + 1));
        }
      }
      int64_t persisted = static_cast<int64_t>(s->received);
      if (a >= 0) {
        if (a > persisted)
          return respond(c_, 400, {}, json_error(400, "Invalid request: missing bytes before offset", "invalid"));
        uint64_t skip = static_cast<uint64_t>(persisted - a);
        if (r.deferred) {
          // stream the chunk: 1 MiB socket reads, CRC'd (and kept) while the
          // client is still sending the rest
          if (piece_.empty()) piece_.resize(1u << 20);
          while (r.deferred) {
            size_t k = static_cast<size_t>(std::min<uint64_t>(r.deferred, piece_.size()));
            bc_.read_exact(piece_.data(), k);
            r.deferred -= k;
            if (skip >= k) {
              skip -= k;
              continue;
            }
            s->append(piece_.data() + skip, k - skip);
            skip = 0;
          }
        } else if (skip < r.body.size()) {
          s->append(r.body.data() + skip, r.body.size() - skip);
        }
        (void)b;
        persisted = static_cast<int64_t>(s->received);
      }
      if (total >= 0 && persisted == total) {
        // the object's CRC32C may come with the final request instead of the
        // session's metadata (x-goog-hash: crc32c=...)
        if (const auto* gh = r.header("x-goog-hash")) {
          bool has = false;
          uint32_t crc = 0;
          std::string md5;
          parse_goog_hash(*gh, &has, &crc, &md5);
          if (has) {
            s->has_crc = true;
            s->crc = crc;
          }
        }
        std::string err;
        auto o = srv_.store().finalize_upload(*s, &err);
        if (!o) return respond(c_, 400, {}, json_error(400, err, "invalid"));
        return respond(c_, 200, {}, object_json(*o, false).dump());
      }
      Headers h;
      if (persisted > 0) h.emplace_back("Range", "bytes=0-" + std::to_string(persisted - 1));
      return respond(c_, 308, h, "", "text/plain");
    }
    respond(c_, 400, {}, json_error(400, "unsupported upload request", "invalid"));
  }

  FakeGcsServer& srv_;
  BufferedConn& bc_;
  std::string body_buf_;
  std::vector<uint8_t> piece_;
  Conn& c_;
};

}  // namespace

void FakeGcsServer::serve_http1(std::unique_ptr<BufferedConn> bc) {
  Http1Handler h(*this, *bc);
  h.run();
}

}  // namespace gcsb
