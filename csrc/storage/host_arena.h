// A receive arena in plain host memory and a sink that takes its payload in
// place: the CPU twin of the GPU connection ring's arena mode
// (gpu/engine.h ConnRing + GpuSink::commit_inplace).  The connection's reader
// recv()s a slot's worth at a time straight into the arena, across HTTP/2
// frame and gRPC message boundaries (net/buffered.h RecvArena); the sink
// copies each payload run out to its object buffer and checks every
// message's CRC32C and the object's on the host.  Used by the CPU tests of
// the arena parse path and by `arena_read` (bindings), not by the benches.
#pragma once
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "net/buffered.h"
#include "storage/sink.h"

namespace gcsb {

class HostArena : public RecvArena {
 public:
  HostArena(size_t slot_bytes, int slots);
  std::pair<uint8_t*, size_t> recv_window() override;
  void received(size_t n) override;
  // the slot currently being filled [base, base + used)
  bool contains(const uint8_t* p, size_t n) const;
  uint64_t recvs() const { return recvs_; }
  uint64_t bytes() const { return bytes_; }
  size_t slot_bytes() const { return slot_bytes_; }

 private:
  size_t slot_bytes_;
  std::vector<uint8_t> mem_;
  int slots_;
  int cur_ = -1;
  size_t used_ = 0;
  uint64_t recvs_ = 0, bytes_ = 0;
};

class InplaceHostSink : public Sink {
 public:
  explicit InplaceHostSink(HostArena* arena) : arena_(arena) {}
  void begin(const ObjectInfo& info) override;
  void update_info(const ObjectInfo& info) override;
  Window acquire(size_t want) override;
  void commit(size_t n) override;
  bool accepts_inplace() const override { return arena_ != nullptr; }
  void commit_inplace(const uint8_t* p, size_t n) override;
  void chunk_begin(size_t len) override;
  void chunk_end(bool has_crc, uint32_t crc) override;
  void resume_at(int64_t offset) override;
  SinkResult finish() override;
  const std::vector<uint8_t>& data() const { return data_; }
  uint64_t inplace_commits() const { return inplace_; }
  uint64_t chunks_checked() const { return chunks_checked_; }

 private:
  void land(const uint8_t* p, size_t n);
  HostArena* arena_;
  ObjectInfo info_;
  std::vector<uint8_t> data_;
  std::vector<uint8_t> window_;  // acquire/commit path (a transport without an arena)
  uint64_t inplace_ = 0, chunks_checked_ = 0;
  uint32_t chunk_crc_ = 0;
  uint64_t chunk_len_ = 0;
  bool in_chunk_ = false, chunk_broken_ = false, mismatch_ = false;
  std::string detail_;
};

}  // namespace gcsb
