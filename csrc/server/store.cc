#include "server/store.h"

#include <openssl/evp.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

#include "core/content.h"
#include "core/crc32c.h"
#include "core/util.h"

namespace gcsb {

Blob::~Blob() {
  if (p_) ::munmap(p_, cap_);
}

void Blob::reserve(size_t n) {
  if (n <= cap_) return;
  const size_t huge = 2u << 20;
  size_t cap = std::max<size_t>(huge, (n + huge - 1) / huge * huge);
  void* q = p_ ? ::mremap(p_, cap_, cap, MREMAP_MAYMOVE)
               : ::mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (q == MAP_FAILED) throw std::bad_alloc();
  ::madvise(q, cap, MADV_HUGEPAGE);
  p_ = static_cast<uint8_t*>(q);
  cap_ = cap;
}

uint8_t* Blob::extend(size_t n) {
  if (size_ + n > cap_) reserve(std::max(size_ + n, cap_ * 2));
  uint8_t* q = p_ + size_;
  size_ += n;
  return q;
}

void Blob::append(const void* p, size_t n) {
  if (n) std::memcpy(extend(n), p, n);
}

const uint8_t* StoredObject::bytes(uint64_t off, uint64_t n) const {
  if (hollow) throw std::runtime_error("object content was not retained by the server (retain_uploads=false)");
  if (synthetic) return PatternBuffer::instance().slice(rot, off, n);
  return data->data() + off;
}

const uint8_t* StoredObject::splice_bytes(uint64_t off, uint64_t n) const {
  if (!synthetic) return nullptr;
  const PatternBuffer& pb = PatternBuffer::instance();
  const uint8_t* t = pb.thp();
  if (!t) return nullptr;
  return t + (pb.slice(rot, off, n) - pb.data());
}

bool StoredObject::file_range(uint64_t off, int* fd, uint64_t* foff) const {
  if (!synthetic) return false;
  const PatternBuffer& pb = PatternBuffer::instance();
  int f = pb.memfd();
  if (f < 0) return false;
  *fd = f;
  *foff = pb.file_offset(rot, off);
  return true;
}

uint32_t StoredObject::crc32c_range(uint64_t off, uint64_t n) const {
  if (hollow) throw std::runtime_error("object content was not retained by the server (retain_uploads=false)");
  if (synthetic) return PatternBuffer::instance().crc32c_range(rot, off, n);
  return gcsb::crc32c(data->data() + off, n);
}

int64_t ObjectStore::next_generation() {
  std::lock_guard<std::mutex> lk(gen_mu_);
  int64_t g = wall_ns() / 1000;
  if (g <= last_gen_) g = last_gen_ + 1;
  last_gen_ = g;
  return g;
}

static std::string md5_of_object(const StoredObject& o);

const std::string& StoredObject::md5() const {
  if (md5_lazy_)
    std::call_once(md5_once_, [this] {
      md5_ = md5_of_object(*this);
      md5_done_.store(true, std::memory_order_release);
    });
  return md5_;
}

static std::string md5_of_object(const StoredObject& o) {
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  EVP_DigestInit_ex(ctx, EVP_md5(), nullptr);
  uint64_t off = 0;
  while (off < o.size) {
    uint64_t n = std::min<uint64_t>(o.size - off, 8 << 20);
    EVP_DigestUpdate(ctx, o.bytes(off, n), n);
    off += n;
  }
  unsigned char md[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  EVP_DigestFinal_ex(ctx, md, &len);
  EVP_MD_CTX_free(ctx);
  return std::string(reinterpret_cast<char*>(md), len);
}

std::shared_ptr<const StoredObject> ObjectStore::get(const std::string& bucket, const std::string& name) const {
  std::shared_lock<std::shared_mutex> lk(mu_);
  auto it = objects_.find({bucket, name});
  return it == objects_.end() ? nullptr : it->second;
}

std::shared_ptr<const StoredObject> ObjectStore::add_synthetic(const std::string& bucket, const std::string& name,
                                                               uint64_t size) {
  auto o = std::make_shared<StoredObject>();
  o->bucket = bucket;
  o->name = name;
  o->size = size;
  o->synthetic = true;
  o->rot = object_rotation(name);
  o->generation = next_generation();
  o->created_us = wall_ns() / 1000;
  o->crc32c = PatternBuffer::instance().crc32c_range(o->rot, 0, size);
  if (compute_md5_) o->set_md5(md5_of_object(*o));
  std::unique_lock<std::shared_mutex> lk(mu_);
  objects_[{bucket, name}] = o;
  return o;
}

void ObjectStore::add_synthetic_range(const std::string& bucket, const std::string& prefix, const std::string& suffix,
                                      int first, int count, uint64_t size) {
  PatternBuffer::instance();  // generate once before fanning out
  std::atomic<int> next{0};
  unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (int i = next++; i < count; i = next++)
        add_synthetic(bucket, prefix + std::to_string(first + i) + suffix, size);
    });
  for (auto& x : th) x.join();
}

std::shared_ptr<const StoredObject> ObjectStore::put(const std::string& bucket, const std::string& name,
                                                     Blob data, const std::string& content_type,
                                                     const uint32_t* known_crc) {
  auto o = std::make_shared<StoredObject>();
  o->bucket = bucket;
  o->name = name;
  o->size = data.size();
  o->content_type = content_type.empty() ? "application/octet-stream" : content_type;
  o->generation = next_generation();
  o->created_us = wall_ns() / 1000;
  o->crc32c = known_crc ? *known_crc : gcsb::crc32c(data.data(), data.size());
  o->data = std::make_shared<const Blob>(std::move(data));
  if (compute_md5_) o->set_md5_lazy();
  std::unique_lock<std::shared_mutex> lk(mu_);
  objects_[{bucket, name}] = o;
  return o;
}

std::shared_ptr<const StoredObject> ObjectStore::compose(const std::string& bucket, const std::string& dest,
                                                         const std::vector<std::string>& sources,
                                                         const std::string& content_type, std::string* err) {
  if (sources.empty() || sources.size() > 32) {
    *err = "The number of source components provided (" + std::to_string(sources.size()) +
           ") must be between 1 and 32";
    return nullptr;
  }
  std::vector<std::shared_ptr<const StoredObject>> src;
  uint64_t total = 0;
  uint32_t crc = 0;
  bool hollow = !retain_uploads_;
  for (const auto& n : sources) {
    auto o = get(bucket, n);
    if (!o) {
      *err = "Object " + n + " (in compose source list) not found";
      return nullptr;
    }
    crc = crc32c_combine(crc, o->crc32c, o->size);
    total += o->size;
    hollow = hollow || o->hollow;
    src.push_back(std::move(o));
  }
  auto out = std::make_shared<StoredObject>();
  out->bucket = bucket;
  out->name = dest;
  out->size = total;
  out->content_type = content_type.empty() ? src[0]->content_type : content_type;
  out->generation = next_generation();
  out->created_us = wall_ns() / 1000;
  out->crc32c = crc;
  out->hollow = hollow;
  if (!hollow) {
    Blob data;
    data.reserve(total);
    for (const auto& o : src)
      for (uint64_t off = 0; off < o->size;) {
        uint64_t n = std::min<uint64_t>(o->size - off, 8u << 20);
        data.append(o->bytes(off, n), n);
        off += n;
      }
    out->data = std::make_shared<const Blob>(std::move(data));
    if (compute_md5_) out->set_md5_lazy();
  }
  std::unique_lock<std::shared_mutex> lk(mu_);
  objects_[{bucket, dest}] = out;
  return out;
}

bool ObjectStore::remove(const std::string& bucket, const std::string& name) {
  std::unique_lock<std::shared_mutex> lk(mu_);
  return objects_.erase({bucket, name}) > 0;
}

std::vector<std::shared_ptr<const StoredObject>> ObjectStore::list(const std::string& bucket, const std::string& prefix,
                                                                   const std::string& start_after, size_t max) const {
  std::vector<std::shared_ptr<const StoredObject>> out;
  std::shared_lock<std::shared_mutex> lk(mu_);
  auto it = objects_.lower_bound({bucket, start_after.empty() ? prefix : std::max(prefix, start_after)});
  for (; it != objects_.end() && out.size() < max; ++it) {
    if (it->first.first != bucket) break;
    const std::string& n = it->first.second;
    if (!start_after.empty() && n <= start_after) continue;
    if (n.compare(0, prefix.size(), prefix) != 0) {
      if (n > prefix) break;
      continue;
    }
    out.push_back(it->second);
  }
  return out;
}

size_t ObjectStore::count() const {
  std::shared_lock<std::shared_mutex> lk(mu_);
  return objects_.size();
}

std::shared_ptr<UploadSession> ObjectStore::start_upload(const std::string& bucket, const std::string& name,
                                                         const std::string& content_type, int64_t expected_size) {
  auto s = std::make_shared<UploadSession>();
  std::lock_guard<std::mutex> lk(up_mu_);
  s->id = "up" + std::to_string(++upload_seq_) + "x" + std::to_string(wall_ns() % 1000000007);
  s->bucket = bucket;
  s->name = name;
  s->content_type = content_type;
  s->expected_size = expected_size;
  s->retain = retain_uploads_;
  if (expected_size > 0 && s->retain) s->data.reserve(static_cast<size_t>(expected_size));
  uploads_[s->id] = s;
  return s;
}

std::shared_ptr<UploadSession> ObjectStore::find_upload(const std::string& id) const {
  std::lock_guard<std::mutex> lk(up_mu_);
  auto it = uploads_.find(id);
  return it == uploads_.end() ? nullptr : it->second;
}

std::shared_ptr<const StoredObject> ObjectStore::finalize_upload(UploadSession& s, std::string* err) {
  if (s.finalized) return s.result;
  const uint32_t got = s.data_crc;
  if (s.has_crc) {
    if (got != s.crc) {
      char b[128];
      std::snprintf(b, sizeof(b), "Provided CRC32C \"%08x\" doesn't match calculated CRC32C \"%08x\"", s.crc, got);
      *err = b;
      return nullptr;
    }
  }
  if (s.retain) {
    s.result = put(s.bucket, s.name, std::move(s.data), s.content_type, &got);
  } else {
    auto o = std::make_shared<StoredObject>();
    o->bucket = s.bucket;
    o->name = s.name;
    o->size = s.received;
    o->hollow = true;
    o->content_type = s.content_type.empty() ? "application/octet-stream" : s.content_type;
    o->generation = next_generation();
    o->created_us = wall_ns() / 1000;
    o->crc32c = got;
    std::unique_lock<std::shared_mutex> lk(mu_);
    objects_[{s.bucket, s.name}] = o;
    s.result = o;
  }
  s.data.clear();
  s.finalized = true;
  return s.result;
}

uint32_t ObjectStore::chunk_crc(const StoredObject& o, uint64_t off, uint64_t n, uint64_t chunk) const {
  if (chunk == 0 || off % chunk != 0 || (n != chunk && off + n != o.size)) return o.crc32c_range(off, n);
  std::shared_ptr<std::vector<uint32_t>> v;
  {
    std::lock_guard<std::mutex> lk(crc_mu_);
    auto& slot = chunk_crcs_[{o.bucket, o.name, o.generation, chunk}];
    if (!slot) {
      slot = std::make_shared<std::vector<uint32_t>>();
      uint64_t nch = (o.size + chunk - 1) / chunk;
      slot->resize(nch);
      for (uint64_t i = 0; i < nch; ++i) {
        uint64_t a = i * chunk, len = std::min<uint64_t>(chunk, o.size - a);
        (*slot)[i] = o.crc32c_range(a, len);
      }
    }
    v = slot;
  }
  return (*v)[off / chunk];
}

}  // namespace gcsb
