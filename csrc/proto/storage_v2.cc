#include "proto/storage_v2.h"

#include "proto/wire.h"

namespace gcsb::v2 {

using pb::Reader;
using pb::WireType;

std::string bucket_resource(const std::string& bucket) {
  if (bucket.rfind("projects/", 0) == 0) return bucket;
  return "projects/_/buckets/" + bucket;
}

std::string bucket_from_resource(std::string_view r) {
  size_t p = r.rfind("/buckets/");
  if (p == std::string_view::npos) return std::string(r);
  return std::string(r.substr(p + 9));
}

static std::string encode_ts(int64_t s, int32_t ns) {
  std::string o;
  pb::put_int64(&o, 1, s);
  pb::put_int64(&o, 2, ns);
  return o;
}

static void decode_ts(std::string_view b, int64_t* s, int32_t* ns) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (f == 1 && wt == pb::kVarint) *s = static_cast<int64_t>(r.varint());
    else if (f == 2 && wt == pb::kVarint) *ns = static_cast<int32_t>(r.varint());
    else r.skip(wt);
  }
}

std::string encode_checksums(bool has_crc, uint32_t crc, const std::string& md5) {
  std::string o;
  if (has_crc) pb::put_fixed32(&o, 1, crc);
  if (!md5.empty()) pb::put_bytes(&o, 2, md5);
  return o;
}

bool decode_checksums(std::string_view b, bool* has_crc, uint32_t* crc, std::string* md5) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (f == 1 && wt == pb::kI32) {
      *crc = r.fixed32();
      *has_crc = true;
    } else if (f == 2 && wt == pb::kLen) {
      *md5 = std::string(r.bytes());
    } else {
      r.skip(wt);
    }
  }
  return r.ok();
}

std::string encode_object(const Object& o) {
  std::string s;
  pb::put_string(&s, 1, o.name);
  pb::put_string(&s, 2, o.bucket);
  pb::put_int64(&s, 3, o.generation);
  pb::put_int64(&s, 4, o.metageneration);
  pb::put_string(&s, 5, o.storage_class);
  pb::put_int64(&s, 6, o.size);
  pb::put_string(&s, 13, o.content_type);
  if (o.create_time_s) pb::put_message(&s, 14, encode_ts(o.create_time_s, o.create_time_ns));
  if (o.has_crc32c || !o.md5.empty()) pb::put_message(&s, 16, encode_checksums(o.has_crc32c, o.crc32c, o.md5));
  if (o.update_time_s) pb::put_message(&s, 17, encode_ts(o.update_time_s, o.update_time_ns));
  pb::put_string(&s, 27, o.etag);
  return s;
}

bool decode_object(std::string_view b, Object* o) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    switch (f) {
      case 1: o->name = std::string(r.bytes()); break;
      case 2: o->bucket = std::string(r.bytes()); break;
      case 3: o->generation = static_cast<int64_t>(r.varint()); break;
      case 4: o->metageneration = static_cast<int64_t>(r.varint()); break;
      case 5: o->storage_class = std::string(r.bytes()); break;
      case 6: o->size = static_cast<int64_t>(r.varint()); break;
      case 13: o->content_type = std::string(r.bytes()); break;
      case 14: decode_ts(r.bytes(), &o->create_time_s, &o->create_time_ns); break;
      case 16: decode_checksums(r.bytes(), &o->has_crc32c, &o->crc32c, &o->md5); break;
      case 17: decode_ts(r.bytes(), &o->update_time_s, &o->update_time_ns); break;
      case 27: o->etag = std::string(r.bytes()); break;
      default: r.skip(wt);
    }
  }
  return r.ok();
}

std::string encode_read_request(const ReadObjectRequest& q) {
  std::string s;
  pb::put_string(&s, 1, q.bucket);
  pb::put_string(&s, 2, q.object);
  pb::put_int64(&s, 3, q.generation);
  pb::put_int64(&s, 4, q.read_offset);
  pb::put_int64(&s, 5, q.read_limit);
  return s;
}

bool decode_read_request(std::string_view b, ReadObjectRequest* q) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    switch (f) {
      case 1: q->bucket = std::string(r.bytes()); break;
      case 2: q->object = std::string(r.bytes()); break;
      case 3: q->generation = static_cast<int64_t>(r.varint()); break;
      case 4: q->read_offset = static_cast<int64_t>(r.varint()); break;
      case 5: q->read_limit = static_cast<int64_t>(r.varint()); break;
      default: r.skip(wt);
    }
  }
  return r.ok();
}

std::string encode_content_range(const ContentRange& c) {
  std::string s;
  pb::put_int64(&s, 1, c.start);
  pb::put_int64(&s, 2, c.end);
  pb::put_int64(&s, 3, c.complete_length);
  return s;
}

bool decode_content_range(std::string_view b, ContentRange* c) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (wt != pb::kVarint) {
      r.skip(wt);
      continue;
    }
    int64_t v = static_cast<int64_t>(r.varint());
    if (f == 1) c->start = v;
    else if (f == 2) c->end = v;
    else if (f == 3) c->complete_length = v;
  }
  return r.ok();
}

ReadResponseFrame encode_read_response(uint64_t content_len, bool has_crc, uint32_t crc, const std::string* checksums,
                                       const std::string* range, const std::string* metadata) {
  ReadResponseFrame fr;
  fr.content_len = content_len;
  // checksummed_data { content (1), crc32c (2) }
  std::string crc_field;
  if (has_crc) pb::put_fixed32(&crc_field, 2, crc);
  const uint64_t content_field = pb::varint_size((1u << 3) | pb::kLen) + pb::varint_size(content_len) + content_len;
  const uint64_t cd_len = content_field + crc_field.size();
  pb::put_len_header(&fr.head, 1, cd_len);
  pb::put_len_header(&fr.head, 1, content_len);
  fr.tail = crc_field;
  if (checksums) pb::put_message(&fr.tail, 2, *checksums);
  if (range) pb::put_message(&fr.tail, 3, *range);
  if (metadata) pb::put_message(&fr.tail, 4, *metadata);
  return fr;
}

std::string encode_get_request(const GetObjectRequest& q) {
  std::string s;
  pb::put_string(&s, 1, q.bucket);
  pb::put_string(&s, 2, q.object);
  pb::put_int64(&s, 3, q.generation);
  return s;
}

bool decode_get_request(std::string_view b, GetObjectRequest* q) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (f == 1) q->bucket = std::string(r.bytes());
    else if (f == 2) q->object = std::string(r.bytes());
    else if (f == 3) q->generation = static_cast<int64_t>(r.varint());
    else r.skip(wt);
  }
  return r.ok();
}

std::string encode_delete_request(const GetObjectRequest& q) {
  std::string s;
  pb::put_string(&s, 1, q.bucket);
  pb::put_string(&s, 2, q.object);
  pb::put_int64(&s, 4, q.generation);
  return s;
}

bool decode_delete_request(std::string_view b, GetObjectRequest* q) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (f == 1) q->bucket = std::string(r.bytes());
    else if (f == 2) q->object = std::string(r.bytes());
    else if (f == 4) q->generation = static_cast<int64_t>(r.varint());
    else r.skip(wt);
  }
  return r.ok();
}

std::string encode_compose_request(const ComposeObjectRequest& q) {
  std::string s;
  pb::put_message(&s, 1, encode_object(q.destination));
  for (const auto& n : q.sources) {
    std::string so;
    pb::put_string(&so, 1, n);
    pb::put_message(&s, 2, so);
  }
  return s;
}

bool decode_compose_request(std::string_view b, ComposeObjectRequest* q) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (f == 1) {
      if (!decode_object(r.bytes(), &q->destination)) return false;
    } else if (f == 2) {
      Reader so(r.bytes());
      uint32_t g;
      WireType w2;
      std::string name;
      while (so.next(&g, &w2)) {
        if (g == 1) name = std::string(so.bytes());
        else so.skip(w2);
      }
      if (!so.ok()) return false;
      q->sources.push_back(name);
    } else {
      r.skip(wt);
    }
  }
  return r.ok();
}

std::string encode_list_request(const ListObjectsRequest& q) {
  std::string s;
  pb::put_string(&s, 1, q.parent);
  pb::put_int64(&s, 2, q.page_size);
  pb::put_string(&s, 3, q.page_token);
  pb::put_string(&s, 4, q.delimiter);
  pb::put_string(&s, 6, q.prefix);
  return s;
}

bool decode_list_request(std::string_view b, ListObjectsRequest* q) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    switch (f) {
      case 1: q->parent = std::string(r.bytes()); break;
      case 2: q->page_size = static_cast<int32_t>(r.varint()); break;
      case 3: q->page_token = std::string(r.bytes()); break;
      case 4: q->delimiter = std::string(r.bytes()); break;
      case 6: q->prefix = std::string(r.bytes()); break;
      default: r.skip(wt);
    }
  }
  return r.ok();
}

std::string encode_list_response(const ListObjectsResponse& l) {
  std::string s;
  for (const auto& o : l.objects) pb::put_message(&s, 1, encode_object(o));
  for (const auto& p : l.prefixes) pb::put_bytes(&s, 2, p);
  pb::put_string(&s, 3, l.next_page_token);
  return s;
}

bool decode_list_response(std::string_view b, ListObjectsResponse* l) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (f == 1) {
      Object o;
      if (!decode_object(r.bytes(), &o)) return false;
      l->objects.push_back(std::move(o));
    } else if (f == 2) {
      l->prefixes.emplace_back(r.bytes());
    } else if (f == 3) {
      l->next_page_token = std::string(r.bytes());
    } else {
      r.skip(wt);
    }
  }
  return r.ok();
}

std::string encode_write_spec(const WriteObjectSpec& sp) {
  std::string s;
  pb::put_message(&s, 1, encode_object(sp.resource));
  if (sp.object_size >= 0) pb::put_int64_always(&s, 8, sp.object_size);
  return s;
}

static bool decode_write_spec(std::string_view b, WriteObjectSpec* sp) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (f == 1) decode_object(r.bytes(), &sp->resource);
    else if (f == 8) sp->object_size = static_cast<int64_t>(r.varint());
    else r.skip(wt);
  }
  return r.ok();
}

WriteRequestParts encode_write_request(const std::string& upload_id, const std::string* spec, int64_t write_offset,
                                       uint64_t content_len, bool has_crc, uint32_t crc, const std::string* checksums,
                                       bool finish_write) {
  WriteRequestParts p;
  if (!upload_id.empty()) pb::put_bytes(&p.head, 1, upload_id);
  if (spec) pb::put_message(&p.head, 2, *spec);
  pb::put_int64(&p.head, 3, write_offset);
  if (content_len > 0 || has_crc) {
    std::string crc_field;
    if (has_crc) pb::put_fixed32(&crc_field, 2, crc);
    uint64_t content_field = content_len ? pb::varint_size((1u << 3) | pb::kLen) + pb::varint_size(content_len) +
                                               content_len
                                         : 0;
    pb::put_len_header(&p.head, 4, content_field + crc_field.size());
    if (content_len) pb::put_len_header(&p.head, 1, content_len);
    p.tail = crc_field;
  }
  if (checksums) pb::put_message(&p.tail, 6, *checksums);
  pb::put_bool(&p.tail, 7, finish_write);
  return p;
}

bool decode_write_request(std::string_view b, WriteObjectRequestView* w) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    switch (f) {
      case 1: w->upload_id = std::string(r.bytes()); break;
      case 2:
        w->has_spec = true;
        decode_write_spec(r.bytes(), &w->spec);
        break;
      case 3: w->write_offset = static_cast<int64_t>(r.varint()); break;
      case 4: {
        w->has_data = true;
        Reader c(r.bytes());
        uint32_t cf;
        WireType cwt;
        while (c.next(&cf, &cwt)) {
          if (cf == 1 && cwt == pb::kLen) w->content = c.bytes();
          else if (cf == 2 && cwt == pb::kI32) {
            w->content_crc = c.fixed32();
            w->has_content_crc = true;
          } else c.skip(cwt);
        }
        if (!c.ok()) return false;
        break;
      }
      case 6:
        w->has_object_checksums = true;
        decode_checksums(r.bytes(), &w->has_object_crc, &w->object_crc, &w->object_md5);
        break;
      case 7: w->finish_write = r.varint() != 0; break;
      default: r.skip(wt);
    }
  }
  return r.ok();
}

std::string encode_write_status(const WriteStatus& st) {
  std::string s;
  if (st.has_resource) pb::put_message(&s, 2, encode_object(st.resource));
  else pb::put_int64_always(&s, 1, st.persisted_size);
  return s;
}

bool decode_write_status(std::string_view b, WriteStatus* st) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (f == 1) st->persisted_size = static_cast<int64_t>(r.varint());
    else if (f == 2) {
      st->has_resource = true;
      decode_object(r.bytes(), &st->resource);
    } else r.skip(wt);
  }
  return r.ok();
}

std::string encode_start_resumable(const WriteObjectSpec& spec, const std::string* checksums) {
  std::string s;
  pb::put_message(&s, 1, encode_write_spec(spec));
  if (checksums) pb::put_message(&s, 5, *checksums);
  return s;
}

bool decode_start_resumable(std::string_view b, WriteObjectSpec* spec, bool* has_crc, uint32_t* crc) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (f == 1) decode_write_spec(r.bytes(), spec);
    else if (f == 5) {
      std::string md5;
      decode_checksums(r.bytes(), has_crc, crc, &md5);
    } else r.skip(wt);
  }
  return r.ok();
}

std::string encode_upload_id(const std::string& id) {
  std::string s;
  pb::put_string(&s, 1, id);
  return s;
}

bool decode_upload_id(std::string_view b, std::string* id) {
  Reader r(b);
  uint32_t f;
  WireType wt;
  while (r.next(&f, &wt)) {
    if (f == 1) *id = std::string(r.bytes());
    else r.skip(wt);
  }
  return r.ok();
}

}  // namespace gcsb::v2
