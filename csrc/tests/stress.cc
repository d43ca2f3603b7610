// Concurrency stress of the host-side core (transports, server, sliced reads,
// uploads, retries) for sanitizer builds:  make asan  /  make tsan.
// SURVEY.md §4.5 / §5 "Race detection": the reference has real data races
// (Q3 main.go:203, Q14 ssd_test/main.go:80) and never runs -race; this binary
// exercises every shared structure of the C++ core from many threads under
// ASan+UBSan and TSan.  Exit status 0 = every read/write verified.
#include <execinfo.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "core/ceiling.h"
#include "core/content.h"
#include "core/crc32c.h"
#include "server/fakegcs.h"
#include "storage/client.h"
#include "storage/sink.h"
#include "storage/sliced.h"

using namespace gcsb;

namespace {

std::atomic<int> g_fail{0};

void check(bool ok, const std::string& what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what.c_str());
    ++g_fail;
  }
}

ClientConfig client_cfg(const std::string& proto, const std::string& url) {
  ClientConfig c;
  c.protocol = proto;
  c.endpoint = Endpoint::parse(url);
  c.retry.initial_s = 0.001;
  c.retry.max_s = 0.01;
  c.retry.max_attempts = 8;
  c.read_chunk = 256 << 10;
  return c;
}

void readers(StorageClient& cli, const std::string& bucket, int nobj, int threads, int reads) {
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      // gRPC / HTTP/2: deferred host CRC (ops replayed by this thread; the ring wraps)
      DiscardSink sink(cli.config().read_chunk, true, cli.config().protocol != "http");
      for (int i = 0; i < reads; ++i) {
        std::string name = "obj_" + std::to_string((t + i) % nobj);
        try {
          ReadResult rr = cli.read_object(bucket, name, sink);
          check(rr.sink.verified && !rr.sink.crc_mismatch,
                cli.transport_name() + " read " + name + " (attempts " + std::to_string(rr.attempts) + ", bytes " +
                    std::to_string(rr.bytes) + ": " + rr.sink.detail + ")");
        } catch (const std::exception& e) {
          check(false, cli.transport_name() + " read " + name + ": " + e.what());
        }
      }
    });
  for (auto& x : th) x.join();
}

}  // namespace

int main(int argc, char** argv) {
  std::set_terminate([] {
    void* f[64];
    const int n = backtrace(f, 64);
    std::fprintf(stderr, "stress: terminate; backtrace:\n");
    backtrace_symbols_fd(f, n, 2);
    std::abort();
  });
  const int scale = argc > 1 ? std::atoi(argv[1]) : 1;
  auto store = std::make_shared<ObjectStore>(true);
  ServerConfig sc;
  FakeGcsServer srv(sc, store);
  srv.start();
  const std::string bucket = "stress";
  const int nobj = 6;
  for (int i = 0; i < nobj; ++i) store->add_synthetic(bucket, "obj_" + std::to_string(i), (3u << 20) + 4097 * i);
  store->add_synthetic(bucket, "big", 12u << 20);

  // the endpoint's sendfile() send source (ServerConfig::send_vmsplice off):
  // concurrent reads over every transport
  {
    ServerConfig sf;
    sf.send_vmsplice = false;
    FakeGcsServer srv2(sf, store);
    srv2.start();
    for (const char* proto : {"http", "grpc"}) {
      auto cli = make_client(client_cfg(proto, srv2.url()));
      readers(*cli, bucket, nobj, 4, 2);
    }
    srv2.stop();
  }

  // the reference's HTTP/2 receive settings (16 KiB DATA frames, 16 MiB
  // windows): six workers' streams multiplexed on one connection land through
  // the spanning receive (h2/h2_client.h H2DataCursor), whose plans meet the
  // other streams' frames and hand bytes back; then a mid-stream disconnect
  for (const char* proto : {"grpc", "http2"}) {
    ClientConfig fc = client_cfg(proto, srv.url());
    fc.h2_max_frame_size = 0;
    fc.h2_window = 16u << 20;
    auto cli = make_client(fc);
    readers(*cli, bucket, nobj, 6, 2 * scale);
    srv.faults().disconnect_at = (1 << 20) + 16384 * 3 + 11;
    srv.faults().disconnect_count = 1;
    readers(*cli, bucket, nobj, 3, 2);
    srv.faults().disconnect_count = 0;
  }

  // one stream goes silent MID-BODY past the read timeout while the others on
  // its connection keep flowing: that stream alone is cancelled (RST_STREAM,
  // the reader may be inside its dispatch), resumes at its delivered offset
  // on the same connection, and the endpoint's stalled handler wakes later
  // into a cancelled stream (tests/test_gpu_conn_ring.py stalled case, host
  // sinks); then the same at 16 KiB frames
  for (const char* proto : {"http2", "grpc", "grpc-16k"}) {
    const bool small = std::strcmp(proto, "grpc-16k") == 0;
    ClientConfig tc = client_cfg(small ? "grpc" : proto, srv.url());
    if (small) {
      tc.h2_max_frame_size = 0;
      tc.h2_window = 16u << 20;
    }
    // the stall outlasts the starvation allowance (h2_client.h
    // kStarvedWindows) even when the other streams are slow (TSan)
    tc.sock.io_timeout_ms = 150;
    tc.retry.max_attempts = 6;
    auto tcli = make_client(tc);
    for (int round = 0; round < 2 * scale; ++round) {
      srv.faults().stall_at = (1 << 20) + 77 * round;
      srv.faults().stall_ms = 1500;
      srv.faults().stall_count = 1;
      std::vector<std::thread> th;
      for (int t = 0; t < 6; ++t)
        th.emplace_back([&, t] {
          auto sink = std::make_unique<DiscardSink>(tc.read_chunk, true, true);
          for (int i = 0; i < 2; ++i) {
            const std::string name = "obj_" + std::to_string((t + i) % nobj);
            try {
              ReadResult rr = tcli->read_object(bucket, name, *sink);
              check(rr.sink.verified && !rr.sink.crc_mismatch,
                    std::string(proto) + " stalled-stream read " + name + ": " + rr.sink.detail);
            } catch (const std::exception& e) {
              check(false, std::string(proto) + " stalled-stream read " + name + ": " + e.what());
            }
          }
        });
      for (auto& x : th) x.join();
    }
    srv.faults().stall_count = 0;
    check(tcli->stats().retries > 0, std::string(proto) + " stalled stream retried");
  }
  // let the last stalled handler wake into its cancelled stream while the
  // endpoint still serves
  std::this_thread::sleep_for(std::chrono::milliseconds(1600));

  // multiplexed reads, plus a mid-stream disconnect on the retry path
  for (const char* proto : {"http2", "grpc"}) {
    ClientConfig rc = client_cfg(proto, srv.url());
    auto cli = make_client(rc);
    readers(*cli, bucket, nobj, 6, 3 * scale);
    srv.faults().disconnect_at = (2 << 20) + 5;
    srv.faults().disconnect_count = 1;
    readers(*cli, bucket, nobj, 4, 2);
    srv.faults().disconnect_count = 0;
  }

  for (const char* proto : {"http", "http2", "grpc"}) {
    auto cli = make_client(client_cfg(proto, srv.url()));
    // 1) many concurrent readers on one client (gRPC: streams multiplexed on one connection)
    readers(*cli, bucket, nobj, 6, 4 * scale);
    // 2) faults while reading: 503s, a mid-stream disconnect, a corrupted byte
    srv.faults().fail_next = 2;
    srv.faults().disconnect_at = (1 << 20) + 3;
    srv.faults().disconnect_count = 1;
    readers(*cli, bucket, nobj, 4, 2);
    srv.faults().disconnect_count = 0;
    srv.faults().corrupt_at = 777;
    srv.faults().corrupt_count = 1;
    {
      DiscardSink s(256 << 10, true, std::string(proto) != "http");
      ReadResult rr = cli->read_object(bucket, "obj_0", s);
      check(rr.sink.crc_mismatch, std::string(proto) + " corruption detected");
    }
    srv.faults().corrupt_count = 0;
    // 3) sliced reads from two threads at once: fixed shares (t=0) and
    //    dynamic 2 MiB pieces pulled from the shared cursor (t=1)
    std::vector<std::thread> th;
    for (int t = 0; t < 2; ++t)
      th.emplace_back([&, t] {
        SlicedReadConfig c;
        c.slices = 4;
        c.min_slice_bytes = 1 << 20;
        c.piece_bytes = t == 1 ? (2u << 20) : 0;
        SlicedReader sr(
            client_cfg(proto, srv.url()), c, [](int) { return std::make_unique<DiscardSink>(256 << 10, true); },
            [](uint64_t) {}, [](int, Sink&, uint64_t, uint64_t) {});
        for (int i = 0; i < 2 * scale; ++i) {
          ReadResult rr = sr.read(bucket, "big");
          check(rr.sink.verified && rr.bytes == (12u << 20), std::string(proto) + " sliced read");
        }
      });
    // 4) concurrent uploads (resumable + simple) and read-back
    for (int t = 0; t < 3; ++t)
      th.emplace_back([&, t] {
        std::vector<uint8_t> data((1u << 20) + 333 * t);
        for (size_t i = 0; i < data.size(); ++i) data[i] = static_cast<uint8_t>(i * 131 + t);
        HostByteSource src(data.data(), data.size());
        WriteOptions wo;
        wo.resumable = t != 1;
        wo.chunk_bytes = 256 << 10;
        std::string name = std::string("up_") + proto + std::to_string(t);
        ObjectMeta m = cli->write_object(bucket, name, src, wo);
        check(m.size == static_cast<int64_t>(data.size()) && m.crc32c == crc32c(data.data(), data.size()),
              std::string(proto) + " upload " + name);
        DiscardSink s(256 << 10, true);
        ReadResult rr = cli->read_object(bucket, name, s);
        check(rr.sink.verified, std::string(proto) + " read-back " + name);
      });
    // 5) listing while everything else runs
    th.emplace_back([&] {
      for (int i = 0; i < 5; ++i) {
        auto all = cli->list_all(bucket, "obj_", 2);
        check(all.size() == static_cast<size_t>(nobj), std::string(proto) + " list");
      }
    });
    for (auto& x : th) x.join();
    // 6) -read-timeout: the endpoint stalls every response for a while, so
    //    concurrent attempts time out, close the shared connection (several
    //    at once on gRPC / HTTP/2), retry and resume once it recovers
    {
      ClientConfig tc = client_cfg(proto, srv.url());
      tc.sock.io_timeout_ms = 30;
      tc.retry.max_attempts = 0;
      tc.retry.max_total_s = 5.0;
      auto tcli = make_client(tc);
      srv.faults().latency_ms = 80;
      std::thread heal([&] {
        std::this_thread::sleep_for(std::chrono::milliseconds(150));
        srv.faults().latency_ms = 0;
      });
      readers(*tcli, bucket, nobj, 4, 2);
      heal.join();
      check(tcli->stats().retries > 0, std::string(proto) + " read timeouts retried");
    }
  }
  srv.stop();
  // 7) the ceiling probe's sender and receiver threads: the THP-object
  //    sender, and an external source staged per read (as the upload bound's
  //    GpuByteSource, here a host copy into two slots) whose pages must stay
  //    put until the receiver has every byte
  {
    CeilingConfig cc;
    cc.object_bytes = 6u << 20;
    cc.reads = 3;
    cc.ring_bytes = 2u << 20;
    cc.recv_chunk = 256u << 10;
    CeilingResult r = tcp_ceiling(cc);
    check(r.gbps > 0, "ceiling probe (THP source)");
    struct Staged : CeilingSource {
      std::vector<uint8_t> obj, stage;
      size_t pos = 0;
      int begins = 0, ends = 0;
      void begin() override {
        ++begins;
        stage.assign(obj.begin(), obj.end());  // "D2H": a fresh copy per read
        pos = 0;
      }
      std::pair<const uint8_t*, size_t> next(size_t max) override {
        const size_t k = std::min(max, stage.size() - pos);
        pos += k;
        return {stage.data() + pos - k, k};
      }
      void end() override {
        ++ends;
        stage.assign(stage.size(), 0);  // reused at once: the receiver must have had every byte
      }
    } src;
    src.obj.resize(cc.object_bytes);
    for (size_t i = 0; i < src.obj.size(); ++i) src.obj[i] = static_cast<uint8_t>(i * 7 + 1);
    cc.source = &src;
    r = tcp_ceiling(cc);
    check(r.gbps > 0 && src.begins == cc.reads && src.ends == cc.reads, "ceiling probe (staged source)");
  }
  if (g_fail) {
    std::fprintf(stderr, "stress: %d failures\n", g_fail.load());
    return 1;
  }
  std::printf("stress: ok\n");
  return 0;
}
