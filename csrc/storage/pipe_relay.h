// Multiplexed receive without the reader's copy: splice() + per-stream pipes.
//
// On one HTTP/2 connection every stream's DATA arrives on one socket, and one
// reader thread must take it off in order.  When that thread recv()s each
// payload into its stream's sink it makes every byte's kernel copy itself, so
// one core bounds the whole connection: config 3 (8 workers, gRPC pool 1)
// and the reference's 48-worker experiment found 4-5 MiB queued on the socket
// at every payload recv() (profiles/r3_w48_tail/recvdiag), with the reader at
// 0.06-0.08 CPU-s/GiB against 0.048 for the one-stream headline.
//
// A PipeRelay stands between that reader and one read's sink.  The reader
// splice()s payload bytes from the socket into the read's pipe -- the kernel
// moves page references of the socket buffers, it copies nothing -- and queues
// the byte count, in order with the sink calls (chunk boundaries, object
// metadata) it would otherwise have made.  The read's own worker thread, which
// waits for the stream anyway (GrpcCall::wait_ok), replays the queue in
// drain(): it read()s the bytes out of the pipe into the real sink's windows
// (the one copy, now on the worker's core) and makes the sink calls.  So a
// connection's streams are copied by as many cores as there are workers,
// and the reader only parses frames and moves pages.
//
// When the pipe is full (its worker is behind) the reader does not wait: it
// recv()s that payload piece into an overflow block (the copy it made before)
// and queues the block's range instead.  Plain TCP only (TLS records must be
// decrypted in user space).
//
// Reference: the Go library reads each gRPC stream's messages on the calling
// goroutine (reference main.go:134-140 io.Copy through the reader), with
// grpc-go's one transport reader per connection copying frames off the
// socket (main.go:30,111 pool size 1); this is the native counterpart of that
// split, with the copy moved to the stream's owner.
#pragma once
#include <sys/types.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "net/buffered.h"
#include "storage/sink.h"

namespace gcsb {

// Process-wide pool of pipes for PipeRelay.  Each pipe is grown to 1 MiB
// (fs.pipe-max-size, the unprivileged limit) or the most the user's pipe
// budget allows; at most kMaxPipes exist at once, so the relays of one
// process stay within a fixed share of the user's pipe pages (fs.pipe-user-
// pages-soft, counted per user across the node's ranks).
struct RelayPipe {
  int r = -1, w = -1;
  size_t cap = 0;
};
struct PipeRelayStats {
  uint64_t relays = 0, no_pipe = 0;       // reads relayed / reads that found no pipe (direct path)
  uint64_t spliced_bytes = 0, splices = 0;
  uint64_t buffered_bytes = 0;            // bytes the reader had already buffered (written into the pipe)
  uint64_t overflow_bytes = 0, overflows = 0;  // pipe full: recv()d into an overflow block
  uint64_t pipes = 0;                     // pipes created
  uint64_t pipe_bytes = 0;                // capacity of the pipes created
};
PipeRelayStats pipe_relay_stats();

class PipeRelay : public Sink {
 public:
  static constexpr size_t kMinPipe = 256 << 10;  // a smaller pipe overflows too often to pay
  static constexpr int kMaxPipes = 64;

  explicit PipeRelay(Sink& inner);
  ~PipeRelay() override;
  PipeRelay(const PipeRelay&) = delete;
  PipeRelay& operator=(const PipeRelay&) = delete;
  // false: no pipe could be had (pool exhausted, user pipe budget); the
  // caller keeps the direct path and must not use this relay.
  bool usable() const { return pipe_.r >= 0; }
  // Sink errors met while replaying (the worker's thread) are reported here,
  // as the direct path reports them from the reader (the read then fails).
  void set_on_error(std::function<void(const std::string&)> f) { on_error_ = std::move(f); }

  // Reader thread: moves 1..n payload bytes from bc into the relay and queues
  // them.  Returns the bytes taken; 0 on orderly EOF.
  size_t feed(BufferedConn& bc, size_t n);

  // Reader thread: queued in order with the payload.
  void update_info(const ObjectInfo& info) override;
  void chunk_begin(size_t len) override;
  void chunk_end(bool has_crc, uint32_t crc) override;
  // The payload goes through feed(); a reader must not ask for windows.
  Window acquire(size_t want) override;
  void commit(size_t n) override;
  // The HTTP/2 media GET begins the sink on the reader (at its response
  // headers): queued like the rest.
  void begin(const ObjectInfo& info) override;
  // Resume / finish / abort belong to the worker and go to the inner sink
  // directly (the read loop calls them outside any stream).
  void resume_at(int64_t offset) override { inner_.resume_at(offset); }
  SinkResult finish() override;
  void abort() override;

  // Worker thread: replays everything queued so far (pipe -> inner sink).
  void drain() override;
  bool deferred() const override { return true; }

  // Worker thread, after the stream is over (the reader no longer feeds this
  // relay): replay what is left, hand overflow blocks and the pipe back.
  void settle();

 private:
  struct Op {
    enum Kind : uint8_t { kPipe, kCopy, kRelease, kOpen, kInfo, kBegin, kEnd } kind;
    bool has_crc = false;
    uint32_t crc = 0;
    size_t len = 0;
    uint8_t* p = nullptr;  // kCopy: bytes in an overflow block; kRelease: the block
    ObjectInfo info;       // kOpen, kInfo
  };
  void push(Op op);
  void apply(const Op& op);
  void deliver(const uint8_t* src, size_t n);  // kCopy into the inner sink
  void pipe_into_sink(size_t n);               // kPipe
  void fail(const char* what);
  size_t read_pipe(uint8_t* dst, size_t n);

  Sink& inner_;
  RelayPipe pipe_;
  std::atomic<bool> pipe_dirty_{false};  // a pipe read failed: bytes of unknown count left in it
  std::function<void(const std::string&)> on_error_;
  // reader side
  uint8_t* blk_ = nullptr;  // overflow block being filled
  size_t blk_used_ = 0;
  std::atomic<int> blocks_{0};  // overflow blocks not yet handed back
  // queue
  std::mutex qmu_;
  std::vector<Op> ops_;
  // worker side
  std::mutex cmu_;
  std::vector<Op> batch_;
  bool failed_ = false;
  std::vector<uint8_t> scratch_;  // pipe bytes a failed sink no longer takes
};

}  // namespace gcsb
