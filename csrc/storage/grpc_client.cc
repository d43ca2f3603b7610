#include "storage/client.h"
#include "core/util.h"
namespace gcsb {
std::unique_ptr<StorageClient> make_grpc_client(const ClientConfig&) {
  throw StorageError("grpc transport not built yet", false);
}
}  // namespace gcsb
