// HTTP/2 client connection: one reader thread demultiplexes frames to
// streams; any thread may open streams and send.  DATA payloads are handed to
// the owning stream *on the socket* (the stream recv()s them straight into its
// destination, e.g. a pinned ring slot), so a multiplexed connection still
// copies each object byte exactly once.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "h2/h2.h"
#include "net/socket.h"

namespace gcsb {

class H2ClientStream {
 public:
  virtual ~H2ClientStream() = default;
  // Response headers or trailers (end_stream set on trailers / trailers-only).
  virtual void on_headers(const HeaderList& h, bool end_stream) = 0;
  // Must consume exactly n bytes from bc (already stripped of padding).
  virtual void on_data(BufferedConn& bc, uint32_t n, bool end_stream) = 0;
  virtual void on_reset(uint32_t code) = 0;
  virtual void on_conn_error(const std::string& msg) = 0;
  uint32_t id() const { return id_; }
  // Frames the reader thread has handed this stream (bumped before and after
  // each dispatch): an idle watchdog compares two samples.
  uint64_t progress() const { return progress_.load(std::memory_order_relaxed); }

  // cv.wait(lk, pred) with an idle limit: idle_ms > 0 gives up once the
  // stream saw no frame for a whole idle_ms window (so after idle_ms to
  // 2 x idle_ms of silence) and returns false; lk is held throughout.
  // A window in which the connection delivered other streams' frames counts
  // as progress up to kStarvedWindows times in a row: on a busy multiplexed
  // connection a stream can wait behind its neighbours' frames (2 MiB gRPC
  // messages) without its server having stalled.
  static constexpr int kStarvedWindows = 3;
  template <class Pred>
  bool wait_progress(std::condition_variable& cv, std::unique_lock<std::mutex>& lk, Pred pred, int idle_ms) {
    if (idle_ms <= 0) {
      cv.wait(lk, pred);
      return true;
    }
#if defined(__SANITIZE_THREAD__)
    // gcc 11's TSan does not intercept pthread_cond_clockwait (steady-clock
    // waits), misses the unlock inside the wait and reports the notifier's
    // lock as a double lock; system-clock deadlines use pthread_cond_timedwait
    using Clock = std::chrono::system_clock;
#else
    using Clock = std::chrono::steady_clock;
#endif
    uint64_t seen = progress();
    uint64_t conn_seen = conn_frames();
    int starved = 0;
    for (;;) {
      if (cv.wait_until(lk, Clock::now() + std::chrono::milliseconds(idle_ms), pred)) return true;
      const uint64_t now = progress(), conn_now = conn_frames();
      if (now != seen) {
        seen = now;
        conn_seen = conn_now;
        starved = 0;
        continue;
      }
      if (conn_now == conn_seen || ++starved > kStarvedWindows) return false;
      conn_seen = conn_now;
    }
  }

 private:
  friend class H2ClientConn;
  uint32_t id_ = 0;
  std::atomic<uint64_t> progress_{0};
  // frames the connection's reader has read (any stream); set by start_stream
  const std::atomic<uint64_t>* conn_frames_ = nullptr;
  uint64_t conn_frames() const { return conn_frames_ ? conn_frames_->load(std::memory_order_relaxed) : 0; }
  // reader dispatches into this stream in flight (taken under the
  // connection's stream-map lock, so none starts once the stream is erased)
  std::atomic<int> busy_{0};
  bool cancelled_ = false;  // cancel_stream() ran (owner thread only)
  RecvWindow recv_window_{16 << 20};
};

struct H2ClientOptions {
  SocketOptions sock;
  uint32_t initial_window = 0x7FFFFFFF;    // per-stream receive window we advertise
  uint32_t max_frame_size = (1u << 24) - 1;  // largest DATA frame we accept
  uint32_t header_table_size = 4096;
  std::vector<int> cpus;  // pin the connection's reader thread
  // receive into this arena (net/buffered.h): the GPU sink's connection ring
  RecvArena* recv_arena = nullptr;
};

// Where the connection reader threads' time goes (process totals): waiting
// for / reading frame headers, dispatching DATA into streams (the receive
// copy), and HEADERS (HPACK decode + completion).  Multiplexed gRPC reads are
// bound by one reader thread per connection, so this is their profile.
struct H2ReaderStats {
  uint64_t frames = 0, data_frames = 0, header_blocks = 0;
  uint64_t data_bytes = 0;
  uint64_t header_wait_ns = 0;  // inside read_frame_header (includes blocking for data)
  uint64_t data_ns = 0;         // DATA frames: stream dispatch incl. recv() into the sink
  uint64_t headers_ns = 0;      // HEADERS/CONTINUATION: read + HPACK decode + stream dispatch
  uint64_t other_ns = 0;        // every other frame type
  // waits over 5 ms for the next frame (an idle connection's first frame
  // after a pause, e.g. a pooled connection reused by a later block): count
  // and their time, so a block's split can leave them out
  uint64_t long_waits = 0, long_wait_ns = 0;
  uint64_t readers_alive = 0;   // connection reader threads running now
};
H2ReaderStats h2_reader_stats();

class H2ClientConn {
 public:
  static std::shared_ptr<H2ClientConn> dial(const Endpoint& ep, const H2ClientOptions& opt);
  ~H2ClientConn();
  // Registers the stream, assigns its id and sends the request headers.
  // Throws StorageError(retryable) if the connection is unusable.
  void start_stream(const std::shared_ptr<H2ClientStream>& s, const HeaderList& headers, bool end_stream);
  // Opens a stream whose whole request body is `body` (END_STREAM on it):
  // HEADERS and DATA leave in one write when they fit one frame each.
  void start_stream_with_body(const std::shared_ptr<H2ClientStream>& s, const HeaderList& headers,
                              const std::string& body);
  // Sends request body bytes honouring flow control (blocks).
  void send_data(H2ClientStream& s, const uint8_t* p, size_t n, bool end_stream);
  void send_data_iov(H2ClientStream& s, struct iovec* iov, int cnt, bool end_stream);
  // Same, from SendPieces (a `splice` piece goes to the socket by page
  // reference, see SendPiece): split into DATA frames by flow control.
  void send_data_pieces(H2ClientStream& s, const std::vector<SendPiece>& pieces, bool end_stream);
  // Forget a stream (RST_STREAM CANCEL if it is still open on our side).
  void end_stream(H2ClientStream& s, bool reset);
  // -read-timeout hit on stream s (its waiter saw no frame for idle_ms).  If
  // the connection itself carried frames within idle_ms, the silence is this
  // stream's: cancel it alone (RST_STREAM, forget it, wait until the reader
  // is outside any dispatch into it) and keep the connection for the other
  // streams multiplexed on it.  If the connection is silent too, or the
  // reader stays inside the stream's dispatch (blocked mid-frame), close the
  // connection.  Either way nothing writes into s's sink afterwards.
  void abandon_stream(H2ClientStream& s, int idle_ms);
  bool usable() const { return !dead_.load() && !goaway_.load(); }
  size_t active_streams();
  const Endpoint& endpoint() const { return ep_; }
  void close();

 private:
  H2ClientConn(Endpoint ep, H2ClientOptions opt) : ep_(std::move(ep)), opt_(opt) {}
  void reader_loop();
  void fail_all(const std::string& msg);
  // the stream with this id, marked busy (release() after the dispatch)
  std::shared_ptr<H2ClientStream> acquire(uint32_t id);
  static void release(H2ClientStream& s) { s.busy_.fetch_sub(1, std::memory_order_release); }
  bool cancel_stream(H2ClientStream& s, int wait_ms);
  Endpoint ep_;
  H2ClientOptions opt_;
  std::unique_ptr<BufferedConn> bc_;
  std::unique_ptr<H2Writer> w_;
  HpackDecoder dec_;
  HpackEncoder enc_;
  std::thread reader_;
  std::mutex close_mu_;  // serialises close()'s join of reader_
  std::mutex mu_;
  std::map<uint32_t, std::shared_ptr<H2ClientStream>> streams_;
  uint32_t next_id_ = 1;
  std::mutex open_mu_;  // id allocation + HEADERS ordering
  H2Settings peer_;
  RecvWindow conn_recv_{64 << 20};
  std::atomic<bool> dead_{false}, goaway_{false};
  std::atomic<int64_t> last_frame_ns_{0};  // steady clock of the last frame header read
  std::atomic<uint64_t> frames_{0};         // frames read (starvation vs stall, H2ClientStream::wait_progress)
  uint32_t goaway_last_ = 0x7FFFFFFF;
  mutable std::mutex reason_mu_;
  std::string dead_reason_;  // guarded by reason_mu_ (written by the reader thread)
  std::string dead_reason() const {
    std::lock_guard<std::mutex> lk(reason_mu_);
    return dead_reason_;
  }
};

}  // namespace gcsb
