// google.storage.v2 message subset used by the benchmark (hand-coded wire
// format; field numbers from the public storage.proto — [lib] per SURVEY.md,
// cross-checked in tests against an independently built descriptor).
//
//   ReadObjectRequest  {bucket=1, object=2, generation=3, read_offset=4, read_limit=5}
//   ReadObjectResponse {checksummed_data=1, object_checksums=2, content_range=3, metadata=4}
//   ChecksummedData    {content=1 bytes, crc32c=2 fixed32}
//   ObjectChecksums    {crc32c=1 fixed32, md5_hash=2 bytes}
//   ContentRange       {start=1, end=2, complete_length=3}
//   Object             {name=1, bucket=2, generation=3, metageneration=4, storage_class=5,
//                       size=6, content_type=13, create_time=14, checksums=16, update_time=17, etag=27}
//   GetObjectRequest   {bucket=1, object=2, generation=3}
//   ListObjectsRequest {parent=1, page_size=2, page_token=3, delimiter=4, prefix=6}
//   ListObjectsResponse{objects=1, prefixes=2, next_page_token=3}
//   WriteObjectSpec    {resource=1, object_size=8}
//   WriteObjectRequest {upload_id=1, write_object_spec=2, write_offset=3, checksummed_data=4,
//                       object_checksums=6, finish_write=7}
//   WriteObjectResponse / QueryWriteStatusResponse {persisted_size=1, resource=2}
//   StartResumableWriteRequest {write_object_spec=1, object_checksums=5}
//   StartResumableWriteResponse{upload_id=1}
//   QueryWriteStatusRequest    {upload_id=1}
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace gcsb::v2 {

constexpr const char* kService = "/google.storage.v2.Storage/";

// "projects/_/buckets/<b>" <-> "<b>"
std::string bucket_resource(const std::string& bucket);
std::string bucket_from_resource(std::string_view r);

struct Object {
  std::string name, bucket, storage_class = "STANDARD", content_type, etag;
  int64_t generation = 0, metageneration = 0, size = 0;
  bool has_crc32c = false;
  uint32_t crc32c = 0;
  std::string md5;
  int64_t create_time_s = 0, update_time_s = 0;
  int32_t create_time_ns = 0, update_time_ns = 0;
};
std::string encode_object(const Object& o);
bool decode_object(std::string_view b, Object* o);

std::string encode_checksums(bool has_crc, uint32_t crc, const std::string& md5);
bool decode_checksums(std::string_view b, bool* has_crc, uint32_t* crc, std::string* md5);

struct ReadObjectRequest {
  std::string bucket, object;  // bucket in resource form
  int64_t generation = 0, read_offset = 0, read_limit = 0;
};
std::string encode_read_request(const ReadObjectRequest& r);
bool decode_read_request(std::string_view b, ReadObjectRequest* r);

struct ContentRange {
  int64_t start = 0, end = 0, complete_length = 0;
};
std::string encode_content_range(const ContentRange& c);
bool decode_content_range(std::string_view b, ContentRange* c);

// The part of a ReadObjectResponse before/after the content bytes, so the
// content itself can be sent with zero copies (writev).
struct ReadResponseFrame {
  std::string head;   // checksummed_data tag+len, content tag+len
  std::string tail;   // crc32c + object_checksums/content_range/metadata
  uint64_t content_len = 0;
};
ReadResponseFrame encode_read_response(uint64_t content_len, bool has_crc, uint32_t crc, const std::string* checksums,
                                       const std::string* range, const std::string* metadata);

struct GetObjectRequest {
  std::string bucket, object;
  int64_t generation = 0;
};
std::string encode_get_request(const GetObjectRequest& r);
bool decode_get_request(std::string_view b, GetObjectRequest* r);

// DeleteObjectRequest {bucket=1, object=2, generation=4} (same fields as Get)
std::string encode_delete_request(const GetObjectRequest& r);
bool decode_delete_request(std::string_view b, GetObjectRequest* r);

// ComposeObjectRequest {destination=1 (Object), source_objects=2 (repeated
// SourceObject {name=1, generation=2})} -> Object
struct ComposeObjectRequest {
  Object destination;  // bucket (resource form) + name + content_type
  std::vector<std::string> sources;
};
std::string encode_compose_request(const ComposeObjectRequest& r);
bool decode_compose_request(std::string_view b, ComposeObjectRequest* r);

struct ListObjectsRequest {
  std::string parent, page_token, delimiter, prefix;
  int32_t page_size = 0;
};
std::string encode_list_request(const ListObjectsRequest& r);
bool decode_list_request(std::string_view b, ListObjectsRequest* r);
struct ListObjectsResponse {
  std::vector<Object> objects;
  std::vector<std::string> prefixes;
  std::string next_page_token;
};
std::string encode_list_response(const ListObjectsResponse& r);
bool decode_list_response(std::string_view b, ListObjectsResponse* r);

struct WriteObjectSpec {
  Object resource;
  int64_t object_size = -1;
};
std::string encode_write_spec(const WriteObjectSpec& s);

// WriteObjectRequest header/trailer around zero-copy content.
struct WriteRequestParts {
  std::string head, tail;
};
// first_upload_id / first_spec: at most one non-empty (first message only).
WriteRequestParts encode_write_request(const std::string& upload_id, const std::string* spec, int64_t write_offset,
                                       uint64_t content_len, bool has_crc, uint32_t crc, const std::string* checksums,
                                       bool finish_write);
struct WriteObjectRequestView {
  std::string upload_id;
  bool has_spec = false;
  WriteObjectSpec spec;
  int64_t write_offset = 0;
  bool has_data = false;
  std::string_view content;
  bool has_content_crc = false;
  uint32_t content_crc = 0;
  bool has_object_checksums = false;
  bool has_object_crc = false;
  uint32_t object_crc = 0;
  std::string object_md5;
  bool finish_write = false;
};
bool decode_write_request(std::string_view b, WriteObjectRequestView* r);

struct WriteStatus {  // WriteObjectResponse / QueryWriteStatusResponse
  bool has_resource = false;
  Object resource;
  int64_t persisted_size = 0;
};
std::string encode_write_status(const WriteStatus& s);
bool decode_write_status(std::string_view b, WriteStatus* s);

std::string encode_start_resumable(const WriteObjectSpec& spec, const std::string* checksums);
bool decode_start_resumable(std::string_view b, WriteObjectSpec* spec, bool* has_crc, uint32_t* crc);
std::string encode_upload_id(const std::string& id);  // StartResumableWriteResponse / QueryWriteStatusRequest
bool decode_upload_id(std::string_view b, std::string* id);

}  // namespace gcsb::v2
