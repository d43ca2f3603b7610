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

class H2ClientConn;

// The DATA frame being dispatched to a stream (H2ClientStream::on_data), on
// the connection's reader thread.  Reads stay inside the frame's payload
// (padding already stripped), except read_spanning(), which may run on into
// the frames that follow.
//
// Why: the reference's grpc-go client (reference go.mod:20, main.go:106-117)
// does not advertise SETTINGS_MAX_FRAME_SIZE, so its peer sends DATA frames
// of at most the RFC 7540 default of 16,384 bytes [lib, parity-unpinned].
// A recv() per 16 KiB frame would bound a 25 GB/s read at its syscall rate,
// so read_spanning() posts ONE recvmsg() whose iovecs predict the wire: the
// rest of this frame's payload, then for each following frame a 9-byte header
// slot and its payload straight after the previous one in dst.  After the
// call every header that arrived is checked (DATA, this stream, no flags,
// the predicted length); the first that is not what the plan assumed ends
// the run and every byte from it on goes back to the parser
// (BufferedConn::unread).  The payload lands contiguously with one kernel
// copy, as with one 2 MiB frame.
class H2DataCursor {
 public:
  uint32_t left() const { return left_; }        // payload bytes of the current frame not read yet
  bool end_stream() const { return end_; }       // END_STREAM on the current frame
  uint32_t stream() const { return stream_; }
  void read_exact(void* dst, size_t n);          // n <= left()
  uint8_t read_byte();
  void skip(size_t n);                           // n <= left()
  size_t read_some(void* dst, size_t n);         // 1..min(n, left()) bytes
  // 1..want payload bytes of this stream into dst, contiguous; may consume
  // following DATA frames of the stream when want > left() (see above).
  size_t read_spanning(uint8_t* dst, size_t want);
  // frames and payload bytes the spanning reads took past the first frame
  uint64_t spanned_frames() const { return spanned_frames_; }

 private:
  friend class H2ClientConn;
  H2DataCursor(BufferedConn& bc, uint32_t stream, uint32_t len, bool end, bool can_span, uint32_t max_frame)
      : bc_(&bc), stream_(stream), left_(len), end_(end), can_span_(can_span), max_frame_(max_frame) {}
  void spill(const struct iovec* iov, int cnt, size_t from_iov, size_t from_off, size_t n);
  BufferedConn* bc_;
  uint32_t stream_;
  uint32_t left_;
  bool end_;
  bool can_span_;
  uint32_t max_frame_;
  uint64_t spanned_frames_ = 0;
  uint64_t spanned_wire_ = 0;  // their frame lengths (flow control)
};

class H2ClientStream {
 public:
  virtual ~H2ClientStream() = default;
  // Response headers or trailers (end_stream set on trailers / trailers-only).
  virtual void on_headers(const HeaderList& h, bool end_stream) = 0;
  // Must consume the whole current frame (c.left() == 0 on return); the
  // frame's END_STREAM is c.end_stream() after the reads (a spanning read
  // moves the cursor to a later frame).
  virtual void on_data(H2DataCursor& c) = 0;
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
  RecvWindow recv_window_{16 << 20};  // threshold set by start_stream from the options
};

struct H2ClientOptions {
  SocketOptions sock;
  // Receive flow control we advertise: the per-stream initial window, and
  // the connection window opened to the same size at dial.  Consumed bytes
  // are credited back (WINDOW_UPDATE) once a quarter of the window is
  // pending, as grpc-go's inFlow does [lib].  grpc-go's BDP estimator grows
  // both windows to at most 16 MiB (its maxWindowSize) [lib, parity-unpinned].
  uint32_t initial_window = 0x7FFFFFFF;
  // Largest DATA frame we accept (SETTINGS_MAX_FRAME_SIZE).  0 = do not
  // advertise: the RFC 7540 default of 16,384 bytes, which is what grpc-go's
  // client leaves its peer with [lib].
  uint32_t max_frame_size = (1u << 24) - 1;
  // DATA frames up to this size are read with H2DataCursor::read_spanning's
  // multi-frame recvmsg(); 0 = never (A/B)
  uint32_t span_max_frame = 256u << 10;
  uint32_t header_table_size = 4096;
  std::vector<int> cpus;  // pin the connection's reader thread
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
  // DATA frames taken by read_spanning past the dispatched one (no header
  // parse of their own on the reader loop), spill = plans whose guess of a
  // frame boundary was wrong
  uint64_t spanned_frames = 0, span_reads = 0, span_spills = 0;
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
  uint32_t accept_max_frame() const { return opt_.max_frame_size ? opt_.max_frame_size : h2::kDefaultMaxFrame; }
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
  RecvWindow conn_recv_{64 << 20};  // threshold reset in dial() from the options
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
