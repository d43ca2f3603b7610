// HTTP/2 (RFC 9113) framing, flow control and connection state shared by the
// native gRPC client (storage/grpc_client.cc) and the fake server
// (server/server_grpc.cc).  Cleartext h2 with prior knowledge ("h2c"), which
// is what a loopback/DirectPath-style endpoint speaks.
//
// Reference: grpc-go's transport (go.mod:20) multiplexes every worker's
// ReadObject stream over ONE HTTP/2 connection when the pool size is 1
// (reference main.go:30,111; SURVEY.md §3.3 "the key contention point").
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "h2/hpack.h"
#include "net/buffered.h"

namespace gcsb {

namespace h2 {
constexpr uint8_t kData = 0x0, kHeaders = 0x1, kPriority = 0x2, kRstStream = 0x3, kSettings = 0x4,
                  kPushPromise = 0x5, kPing = 0x6, kGoaway = 0x7, kWindowUpdate = 0x8, kContinuation = 0x9;
constexpr uint8_t kFlagEndStream = 0x1, kFlagAck = 0x1, kFlagEndHeaders = 0x4, kFlagPadded = 0x8,
                  kFlagPriority = 0x20;
constexpr uint16_t kSettingsHeaderTableSize = 1, kSettingsEnablePush = 2, kSettingsMaxConcurrentStreams = 3,
                   kSettingsInitialWindowSize = 4, kSettingsMaxFrameSize = 5, kSettingsMaxHeaderListSize = 6;
constexpr uint32_t kErrNoError = 0, kErrProtocol = 1, kErrInternal = 2, kErrFlowControl = 3, kErrCancel = 8,
                   kErrRefusedStream = 7;
constexpr int64_t kMaxWindow = 0x7FFFFFFF;
constexpr uint32_t kDefaultWindow = 65535;
constexpr uint32_t kDefaultMaxFrame = 16384;
constexpr uint32_t kMaxFrameLimit = (1u << 24) - 1;
extern const char kPreface[25];  // "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"
}  // namespace h2

struct FrameHeader {
  uint32_t length = 0;
  uint8_t type = 0;
  uint8_t flags = 0;
  uint32_t stream = 0;
};

void encode_frame_header(uint8_t out[9], uint32_t len, uint8_t type, uint8_t flags, uint32_t stream);
FrameHeader read_frame_header(BufferedConn& bc);

struct H2Settings {
  uint32_t header_table_size = 4096;
  uint32_t enable_push = 1;
  uint32_t max_concurrent_streams = 0xFFFFFFFF;
  uint32_t initial_window_size = h2::kDefaultWindow;
  uint32_t max_frame_size = h2::kDefaultMaxFrame;
  uint32_t max_header_list_size = 0xFFFFFFFF;
};

// Payload of a SETTINGS frame.
std::string encode_settings(const std::vector<std::pair<uint16_t, uint32_t>>& kv);

// A payload piece: memory, or a file range sent with sendfile() (zero copy).
struct SendPiece {
  const uint8_t* p = nullptr;
  size_t n = 0;
  int fd = -1;
  uint64_t foff = 0;
  // user memory sent by vmsplice + splice (Conn::splice_user_all): no copy,
  // the pages must stay unchanged until the peer has read them
  bool splice = false;
};

// Mutual exclusion granted in arrival order, one wake per hand-off.  The
// frame writes of a connection's streams go through it: a std::mutex lets
// the thread that just wrote a frame take the lock straight back, so with 48
// streams multiplexed on one connection some waited ~10 ms for their first
// frame.  lock_wait_ns(): how long the last lock() of
// the calling thread waited.
class FifoLock {
 public:
  void lock();
  bool try_lock();  // only when free: never ahead of queued waiters
  void unlock();
  static int64_t last_wait_ns();

 private:
  struct Waiter {
    std::condition_variable cv;
    bool granted = false;
  };
  std::mutex mu_;
  bool held_ = false;
  std::deque<Waiter*> q_;
};

// Frame-write statistics of one H2Writer: DATA frames written and how long
// their writers queued for the connection (the endpoint's per-stream
// fairness, ServerStats::h2_*).
struct H2SendStats {
  std::atomic<uint64_t> data_frames{0}, queue_wait_ns{0}, queue_wait_max_ns{0};
};

// Per-direction connection machinery common to both roles: serialized
// writes, peer settings, send-side flow-control windows.
class H2Writer {
 public:
  explicit H2Writer(Conn& c) : conn_(c) {}
  // While more than one stream is registered, DATA frames are capped at
  // `bytes` (0 = the peer's max frame size only): the streams' frames then
  // interleave in FIFO order at this grain (round-robin over the streams
  // with data ready) instead of one stream's whole message holding the
  // connection.  The endpoint sets 256 KiB (ServerConfig::h2_quantum).
  void set_quantum(size_t bytes) { quantum_ = bytes; }
  // DATA-frame statistics also go to *sink (e.g. the endpoint's totals)
  void set_stats_sink(H2SendStats* sink) { sink_ = sink; }
  const H2SendStats& send_stats() const { return sstats_; }
  // Writes one frame (header + payload pieces) atomically w.r.t. other writers.
  void write_frame(uint8_t type, uint8_t flags, uint32_t stream, const void* p, size_t n);
  void write_frame_iov(uint8_t type, uint8_t flags, uint32_t stream, struct iovec* payload, int cnt, size_t total);
  // lead_headers: a HEADERS block (END_HEADERS) written just before the DATA
  // frame, in its first write; trailers: a HEADERS block (END_STREAM |
  // END_HEADERS) written right after it, in its last write.  A 1 MiB gRPC
  // response is then 4 system calls on the sender (writev, vmsplice, splice,
  // writev) instead of 6, and its trailers no separate loopback segment that
  // wakes the client's reader once more.  Both blocks must fit one frame.
  void write_frame_pieces(uint8_t type, uint8_t flags, uint32_t stream, const std::vector<SendPiece>& pieces,
                          size_t total,
                          const std::string* lead_headers = nullptr, const std::string* trailers = nullptr);
  // A train of DATA frames of one stream in ONE write: `total` payload bytes
  // (send window already reserved, e.g. try_reserve_train) cut into frames
  // of at most the peer's SETTINGS_MAX_FRAME_SIZE, `last_flags` on the last
  // one; lead_headers / trailers as in write_frame_pieces.  Frames below
  // kTrainCopyMaxFrame go as ONE writev of every header and payload piece
  // (the kernel copies the payload; a `splice` piece is read as memory):
  // at the RFC default of 16 KiB -- what a client that advertises no larger
  // SETTINGS_MAX_FRAME_SIZE, grpc-go's, receives -- vmsplice()ing a 9-byte
  // header and 4 pages per frame stalled reads for up to 1.2 s on loopback
  // (5 of 8 reads > 90 ms), one write per 1 MiB of frames did not.  Larger
  // frames keep write_frame_pieces (vmsplice / sendfile per frame), as do
  // `fd` pieces.
  static constexpr size_t kTrainCopyMaxFrame = 256u << 10;
  void write_data_train(uint32_t stream, const std::vector<SendPiece>& pieces, size_t total, uint8_t last_flags,
                        const std::string* lead_headers = nullptr, const std::string* trailers = nullptr);
  // Header block (HEADERS + CONTINUATION as needed).
  void write_headers(uint32_t stream, const std::string& block, bool end_stream);
  // HEADERS + one DATA frame (END_STREAM) in a single writev: a unary or
  // server-streaming request reaches the peer in one segment.  Returns false
  // (nothing written) if the block or the body does not fit one frame / the
  // current send windows; the caller then sends them separately.
  bool write_headers_and_data(uint32_t stream, const std::string& block, const uint8_t* p, size_t n);
  void write_window_update(uint32_t stream, uint32_t inc);
  void write_rst(uint32_t stream, uint32_t code);
  void write_goaway(uint32_t last_stream, uint32_t code, const std::string& msg);
  void write_settings(const std::string& payload) { write_frame(h2::kSettings, 0, 0, payload.data(), payload.size()); }
  void write_settings_ack() { write_control(h2::kSettings, h2::kFlagAck, 0, nullptr, 0); }
  void write_ping_ack(const uint8_t opaque[8]) { write_control(h2::kPing, h2::kFlagAck, 0, opaque, 8); }
  // A control frame from the connection's reader thread (WINDOW_UPDATE,
  // SETTINGS / PING acks): written now if no frame write is in progress,
  // else queued for the writer holding the connection to send before it
  // lets go.  The reader never blocks behind a DATA writer: two peers whose
  // DATA writers each wait for the other's socket to drain keep reading,
  // so their queued WINDOW_UPDATEs still go out (a blocked reader on both
  // ends was a deadlock, made likelier by FIFO hand-off).
  void write_control(uint8_t type, uint8_t flags, uint32_t stream, const void* p, size_t n);

  // --- send flow control ---------------------------------------------------
  // Blocks until the connection and stream windows allow >=1 byte; returns
  // how many bytes (<= want, <= peer max frame) may be sent now and debits
  // them.  Returns 0 if the connection/stream is dead.
  size_t reserve(uint32_t stream, size_t want);
  // reserve() that never blocks: 0 if the windows allow nothing now; *gone
  // set (and 0 returned) if the stream or the connection is dead.
  size_t try_reserve(uint32_t stream, size_t want, bool* gone);
  // reserve() / try_reserve() for a frame train: up to `want` bytes, bounded
  // by the send windows only (write_data_train cuts the frames).  Less than
  // want (window-limited) is rounded down to whole max-size frames when at
  // least one fits, so a message's frames stay full-size up to its last.
  size_t reserve_train(uint32_t stream, size_t want);
  size_t try_reserve_train(uint32_t stream, size_t want, bool* gone);
  // Waits up to timeout_ms for a window update (or kill / settings change).
  void wait_window(int timeout_ms);
  void register_stream(uint32_t stream);
  void unregister_stream(uint32_t stream);
  void on_window_update(uint32_t stream, uint32_t inc);
  void on_peer_settings(const H2Settings& s, uint32_t old_initial_window);
  void kill();  // wake all waiters; further reserve() returns 0
  uint32_t peer_max_frame() const { return peer_max_frame_; }
  uint32_t peer_initial_window() const { return peer_initial_window_; }
  Conn& conn() { return conn_; }

 private:
  void note_data_frame();
  size_t train_grant_locked(int64_t avail, size_t want) const;
  // Holds wmu_ for one frame write; on release sends the control frames
  // queued meanwhile (write_control), then unlocks.
  class WriteLock {
   public:
    explicit WriteLock(H2Writer& w) : w_(w) { w_.wmu_.lock(); }
    ~WriteLock() { w_.release(); }
    WriteLock(const WriteLock&) = delete;
    WriteLock& operator=(const WriteLock&) = delete;

   private:
    H2Writer& w_;
  };
  void release();  // flush queued control frames, unlock wmu_
  Conn& conn_;
  FifoLock wmu_;  // frame writes, granted in arrival order
  std::mutex ctl_mu_;        // guards ctl_pending_; taken before wmu_'s own mutex
  std::string ctl_pending_;  // encoded control frames waiting for the writer
  size_t quantum_ = 0;
  H2SendStats sstats_;
  H2SendStats* sink_ = nullptr;
  std::mutex fmu_;  // flow control
  std::condition_variable fcv_;
  int64_t conn_window_ = h2::kDefaultWindow;
  std::map<uint32_t, int64_t> stream_window_;
  // written by the connection's reader thread (SETTINGS), read by writers
  // that do not hold fmu_ (header blocks are split by the max frame size)
  std::atomic<uint32_t> peer_max_frame_{h2::kDefaultMaxFrame};
  std::atomic<uint32_t> peer_initial_window_{h2::kDefaultWindow};
  bool dead_ = false;
};

// Receive-side window replenishment: credits consumed bytes back to the peer
// once `threshold` of them are pending (a quarter of the advertised window,
// as grpc-go's inFlow [lib]; at most 16 / 64 MiB for the 2^31-1 windows).
class RecvWindow {
 public:
  explicit RecvWindow(int64_t threshold = 64 << 20) : threshold_(threshold) {}
  void set_threshold(int64_t t) { threshold_ = t; }
  // the threshold for an advertised window of w bytes
  static int64_t threshold_for(uint32_t w, int64_t cap) { return std::max<int64_t>(1, std::min<int64_t>(w / 4, cap)); }
  // returns increment to send now (0 = nothing yet)
  uint32_t consume(uint32_t n) {
    pending_ += n;
    if (pending_ >= threshold_) {
      uint32_t inc = static_cast<uint32_t>(pending_);
      pending_ = 0;
      return inc;
    }
    return 0;
  }

 private:
  int64_t threshold_;
  int64_t pending_ = 0;
};

// Parses a SETTINGS payload into s (returns false on malformed payload).
bool apply_settings_payload(const uint8_t* p, size_t n, H2Settings* s);

}  // namespace gcsb
