// Media-read semantics of the synthetic GCS endpoint shared by its HTTP/1.1
// front end (server_http1.cc) and its HTTP/2 front end (server_grpc.cc, plain
// GETs on an h2c connection): which object a path names, the response status
// and headers of a (ranged) media GET, and the JSON bodies both send.
//
// What a real GCS media response carries is what the reference's storage
// library reads: x-goog-hash crc32c/md5 (full-read CRC check),
// x-goog-generation (generation pinning on resume), Content-Range on 206.
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "core/json.h"
#include "server/store.h"

namespace gcsb {

using MediaHeaders = std::vector<std::pair<std::string, std::string>>;

// A request path split into the object it names.
struct MediaTarget {
  enum Kind { kNone, kXml, kJsonMedia, kJsonMeta } kind = kNone;
  std::string bucket, name;
};
// path without the query; alt = the `alt` query parameter.
MediaTarget route_object_path(const std::string& path, const std::string& alt);

// Response of a media GET/HEAD for object o.  status >= 400: body/content_type
// hold the error; else the body is bytes [start, start + len) of the object.
struct MediaPlan {
  int status = 200;
  MediaHeaders headers;  // without Content-Length / Content-Type of errors
  uint64_t start = 0, len = 0;
  std::string body, content_type;
};
// range: the Range header value or nullptr; generation: the `generation`
// query value or nullptr.
MediaPlan plan_media(const StoredObject& o, const std::string* range, const std::string* generation);

// "bytes=a-b" / "bytes=a-" / "bytes=-n" against an object of `size` bytes.
bool parse_byte_range(const std::string& v, uint64_t size, uint64_t* a, uint64_t* b);

std::string json_error(int code, const std::string& msg, const std::string& reason);
Json object_json(const StoredObject& o, bool force_md5 = true);
std::string rfc3339(int64_t us);
std::string http_date(int64_t us);

}  // namespace gcsb
