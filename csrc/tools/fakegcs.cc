// Standalone synthetic GCS endpoint (HTTP/1.1 XML+JSON and h2c gRPC on one
// port).  Used by scripts/execute_pb.sh, the CLI's --start-server option and
// one-process-per-GPU benchmarks (each rank can run its own endpoint).
#include <signal.h>

#include <fstream>
#include <memory>
#include <sstream>

#include "core/util.h"
#include "server/fakegcs.h"
#include "tools/goflags.h"

using namespace gcsb;

int main(int argc, char** argv) {
  GoFlags f("fakegcs");
  auto host = f.String("host", "127.0.0.1", "Listen address");
  auto port = f.Int("port", 0, "Listen port (0 = ephemeral)");
  auto port_file = f.String("port-file", "", "Write the bound port to this file once listening");
  auto bucket = f.String("bucket", "princer-working-dirs", "Bucket holding the synthetic objects");
  auto prefix = f.String("object-prefix", "princer_100M_files/file_", "Synthetic object name prefix");
  auto suffix = f.String("object-suffix", "", "Synthetic object name suffix");
  auto first = f.Int("first-object", 0, "Index of the first synthetic object");
  auto count = f.Int("objects", 48, "Number of synthetic objects prefix<i>suffix");
  auto size = f.Int("object-size", 100 << 20, "Synthetic object size in bytes");
  auto md5 = f.Bool("md5", true, "Compute MD5 for synthetic objects (x-goog-hash md5=)");
  auto retain = f.Bool("retain-uploads", true, "Keep uploaded bytes (false: verify size + CRC32C, keep metadata only)");
  auto require_auth = f.Bool("require-auth", false, "Require a bearer token issued by /token");
  auto jwt_key = f.String("jwt-public-key", "", "PEM public key used to verify JWT assertions at /token");
  auto grpc_chunk = f.Int("grpc-chunk", 2 << 20, "ReadObjectResponse content bytes per message");
  auto fail_next = f.Int("fail-next", 0, "Fail the next N data requests");
  auto fail_status = f.Int("fail-status", 503, "HTTP status for injected failures");
  auto throttle = f.Int("throttle-bps", 0, "Per-response byte rate cap");
  auto latency = f.Int("latency-ms", 0, "Added time to first byte");
  auto tls_cert = f.String("tls-cert", "", "PEM certificate: serve https / gRPC over TLS (ALPN h2)");
  auto tls_key = f.String("tls-key", "", "PEM private key for -tls-cert");
  f.Parse(argc, argv);

  sigset_t set;
  sigemptyset(&set);
  sigaddset(&set, SIGINT);
  sigaddset(&set, SIGTERM);
  pthread_sigmask(SIG_BLOCK, &set, nullptr);

  ServerConfig cfg;
  cfg.host = *host;
  cfg.port = static_cast<int>(*port);
  cfg.require_auth = *require_auth;
  cfg.grpc_chunk = static_cast<uint64_t>(*grpc_chunk);
  cfg.tls_cert_file = *tls_cert;
  cfg.tls_key_file = *tls_key;
  if (!jwt_key->empty()) {
    std::ifstream in(*jwt_key);
    std::stringstream ss;
    ss << in.rdbuf();
    cfg.jwt_public_key_pem = ss.str();
  }
  auto store = std::make_shared<ObjectStore>(*md5);
  store->set_retain_uploads(*retain);
  int64_t t0 = now_ns();
  if (*count > 0)
    store->add_synthetic_range(*bucket, *prefix, *suffix, static_cast<int>(*first), static_cast<int>(*count),
                               static_cast<uint64_t>(*size));
  FakeGcsServer srv(cfg, store);
  srv.faults().fail_next = static_cast<int>(*fail_next);
  srv.faults().fail_status = static_cast<int>(*fail_status);
  srv.faults().throttle_bps = *throttle;
  srv.faults().latency_ms = static_cast<int>(*latency);
  srv.start();
  std::fprintf(stderr, "fakegcs: %lld objects of %lld bytes in gs://%s/%s<i>%s ready in %.2f s; listening on %s\n",
               static_cast<long long>(*count), static_cast<long long>(*size), bucket->c_str(), prefix->c_str(),
               suffix->c_str(), (now_ns() - t0) / 1e9, srv.url().c_str());
  if (!port_file->empty()) {
    std::string tmp = *port_file + ".tmp";
    {
      std::ofstream o(tmp);
      o << srv.port() << "\n";
    }
    std::rename(tmp.c_str(), port_file->c_str());
  }
  int sig = 0;
  sigwait(&set, &sig);
  srv.stop();
  auto& s = srv.stats();
  std::fprintf(stderr, "fakegcs: stopped (signal %d): %llu connections, %llu http requests, %llu grpc calls, %llu bytes sent\n",
               sig, static_cast<unsigned long long>(s.connections.load()),
               static_cast<unsigned long long>(s.http_requests.load()),
               static_cast<unsigned long long>(s.grpc_calls.load()), static_cast<unsigned long long>(s.bytes_sent.load()));
  return 0;
}
