#include "server/media.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>

#include "core/util.h"
#include "storage/client.h"

namespace gcsb {

std::string rfc3339(int64_t us) {
  time_t s = static_cast<time_t>(us / 1000000);
  tm t{};
  gmtime_r(&s, &t);
  char b[64];
  std::snprintf(b, sizeof(b), "%04d-%02d-%02dT%02d:%02d:%02d.%03dZ", t.tm_year + 1900, t.tm_mon + 1, t.tm_mday,
                t.tm_hour, t.tm_min, t.tm_sec, static_cast<int>((us / 1000) % 1000));
  return b;
}

std::string http_date(int64_t us) {
  time_t s = static_cast<time_t>(us / 1000000);
  tm t{};
  gmtime_r(&s, &t);
  char b[64];
  std::strftime(b, sizeof(b), "%a, %d %b %Y %H:%M:%S GMT", &t);
  return b;
}

std::string json_error(int code, const std::string& msg, const std::string& reason) {
  Json e = Json::object();
  Json err = Json::object();
  err.set("code", Json::num(code));
  err.set("message", Json::str(msg));
  Json arr = Json::array();
  Json one = Json::object();
  one.set("message", Json::str(msg));
  one.set("reason", Json::str(reason));
  one.set("domain", Json::str("global"));
  arr.push(one);
  err.set("errors", arr);
  e.set("error", err);
  return e.dump();
}

Json object_json(const StoredObject& o, bool force_md5) {
  Json j = Json::object();
  j.set("kind", Json::str("storage#object"));
  j.set("id", Json::str(o.bucket + "/" + o.name + "/" + std::to_string(o.generation)));
  j.set("selfLink", Json::str("/storage/v1/b/" + o.bucket + "/o/" + url_encode(o.name)));
  j.set("mediaLink", Json::str("/download/storage/v1/b/" + o.bucket + "/o/" + url_encode(o.name) +
                               "?generation=" + std::to_string(o.generation) + "&alt=media"));
  j.set("name", Json::str(o.name));
  j.set("bucket", Json::str(o.bucket));
  j.set("generation", Json::str(std::to_string(o.generation)));
  j.set("metageneration", Json::str(std::to_string(o.metageneration)));
  j.set("contentType", Json::str(o.content_type));
  j.set("storageClass", Json::str("STANDARD"));
  j.set("size", Json::str(std::to_string(o.size)));
  if ((force_md5 || o.md5_ready()) && !o.md5().empty()) j.set("md5Hash", Json::str(base64_encode(o.md5())));
  j.set("crc32c", Json::str(crc32c_b64(o.crc32c)));
  j.set("etag", Json::str("CK" + std::to_string(o.generation % 1000000) + "E="));
  j.set("timeCreated", Json::str(rfc3339(o.created_us)));
  j.set("updated", Json::str(rfc3339(o.created_us)));
  return j;
}

MediaTarget route_object_path(const std::string& path, const std::string& alt) {
  MediaTarget t;
  std::string rest;
  if (starts_with(path, "/storage/v1/b/")) rest = path.substr(std::strlen("/storage/v1/b/"));
  else if (starts_with(path, "/download/storage/v1/b/")) rest = path.substr(std::strlen("/download/storage/v1/b/"));
  if (!rest.empty()) {
    size_t sl = rest.find('/');
    if (sl == std::string::npos || rest.compare(sl, 3, "/o/") != 0 || sl + 3 >= rest.size()) return t;
    t.bucket = url_decode(rest.substr(0, sl));
    t.name = url_decode(rest.substr(sl + 3));
    t.kind = alt == "media" ? MediaTarget::kJsonMedia : MediaTarget::kJsonMeta;
    return t;
  }
  // XML API: /<bucket>/<object>
  if (path.size() < 2 || path[0] != '/') return t;
  std::string p = path.substr(1);
  size_t sl = p.find('/');
  if (sl == std::string::npos || sl + 1 >= p.size()) return t;
  t.bucket = url_decode(p.substr(0, sl));
  t.name = url_decode(p.substr(sl + 1));
  t.kind = MediaTarget::kXml;
  return t;
}

bool parse_byte_range(const std::string& v, uint64_t size, uint64_t* a, uint64_t* b) {
  if (!starts_with(v, "bytes=")) return false;
  std::string s = v.substr(6);
  size_t dash = s.find('-');
  if (dash == std::string::npos) return false;
  std::string x = s.substr(0, dash), y = s.substr(dash + 1);
  char* end = nullptr;
  if (x.empty()) {
    if (y.empty()) return false;
    uint64_t n = std::strtoull(y.c_str(), &end, 10);
    if (*end) return false;
    *a = n >= size ? 0 : size - n;
    *b = size ? size - 1 : 0;
    return true;
  }
  *a = std::strtoull(x.c_str(), &end, 10);
  if (*end) return false;
  if (y.empty()) {
    *b = size ? size - 1 : 0;
  } else {
    uint64_t yb = std::strtoull(y.c_str(), &end, 10);
    if (*end || yb < *a) return false;
    *b = std::min<uint64_t>(yb, size ? size - 1 : 0);
  }
  return true;
}

MediaPlan plan_media(const StoredObject& o, const std::string* range, const std::string* generation) {
  MediaPlan p;
  if (generation && std::strtoll(generation->c_str(), nullptr, 10) != o.generation) {
    p.status = 404;
    p.body = json_error(404, "No such object: " + o.bucket + "/" + o.name + "#" + *generation, "notFound");
    p.content_type = "application/json; charset=UTF-8";
    return p;
  }
  if (o.hollow) {
    p.status = 412;
    p.body = json_error(412, "object content was not retained (server retain_uploads=false)", "conditionNotMet");
    p.content_type = "application/json; charset=UTF-8";
    return p;
  }
  uint64_t a = 0, b = o.size ? o.size - 1 : 0;
  bool partial = false;
  if (range && o.size > 0 && parse_byte_range(*range, o.size, &a, &b)) {
    if (a >= o.size) {
      p.status = 416;
      p.headers.emplace_back("Content-Range", "bytes */" + std::to_string(o.size));
      p.body = json_error(416, "Requested range not satisfiable", "requestedRangeNotSatisfiable");
      p.content_type = "application/json; charset=UTF-8";
      return p;
    }
    partial = true;
  }
  p.status = partial ? 206 : 200;
  p.start = a;
  p.len = o.size ? b - a + 1 : 0;
  p.headers = {{"Content-Type", o.content_type},
               {"Accept-Ranges", "bytes"},
               {"x-goog-generation", std::to_string(o.generation)},
               {"x-goog-metageneration", std::to_string(o.metageneration)},
               {"x-goog-stored-content-length", std::to_string(o.size)},
               {"x-goog-stored-content-encoding", "identity"},
               {"x-goog-storage-class", "STANDARD"},
               {"x-goog-hash", "crc32c=" + crc32c_b64(o.crc32c)},
               {"ETag", "\"" + std::to_string(o.generation) + "\""},
               {"Last-Modified", http_date(o.created_us)},
               {"Server", "gcsb-fakegcs"}};
  if (!o.md5().empty()) p.headers.emplace_back("x-goog-hash", "md5=" + base64_encode(o.md5()));
  if (partial)
    p.headers.emplace_back("Content-Range",
                           "bytes " + std::to_string(a) + "-" + std::to_string(b) + "/" + std::to_string(o.size));
  return p;
}

}  // namespace gcsb
