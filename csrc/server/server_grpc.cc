// h2c gRPC front end of the synthetic GCS server (placeholder until the
// HTTP/2 stack lands).
#include "net/buffered.h"
#include "server/fakegcs.h"

namespace gcsb {
void FakeGcsServer::serve_h2(std::unique_ptr<BufferedConn> bc) { bc->conn().close(); }
}  // namespace gcsb
