// RCCL logits gather behind the C ABI: the one collective of the
// data-parallel eval forward -- each rank's [B/W, classes] fp32 logits to rank 0 over xGMI --
// replacing nn.DataParallel's gather (reference main.py:345).  One process per GPU; the
// communicator is the library's only global mutable state (every entry point holds its mutex).
#include <string.h>

#include <mutex>

#include <rccl/rccl.h>

#include "qnn_internal.h"

namespace qnn {
namespace {
std::mutex g_comm_mu;
ncclComm_t g_comm = nullptr;
int g_rank = -1, g_world = 0;

int nccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return QNN_OK;
  set_error(std::string(what) + ": " + ncclGetErrorString(r));
  return QNN_ERR_HIP;
}
}  // namespace
}  // namespace qnn

using namespace qnn;

extern "C" int qnn_comm_unique_id(void* id, size_t bytes) {
  QNN_REQUIRE(id && bytes >= sizeof(ncclUniqueId), "unique id buffer smaller than QNN_COMM_ID_BYTES");
  ncclUniqueId u;
  const int rc = nccl_check(ncclGetUniqueId(&u), "ncclGetUniqueId");
  if (rc != QNN_OK) return rc;
  memcpy(id, &u, sizeof(u));
  return QNN_OK;
}

extern "C" int qnn_comm_init(int rank, int world, const void* unique_id) {
  QNN_REQUIRE(world >= 1 && rank >= 0 && rank < world, "rank / world out of range");
  QNN_REQUIRE(unique_id, "null unique id");
  std::lock_guard<std::mutex> lock(g_comm_mu);
  QNN_REQUIRE(!g_comm, "communicator already initialised (qnn_comm_destroy first)");
  ncclUniqueId u;
  memcpy(&u, unique_id, sizeof(u));
  ncclComm_t c = nullptr;
  const int rc = nccl_check(ncclCommInitRank(&c, world, u, rank), "ncclCommInitRank");
  if (rc != QNN_OK) return rc;
  g_comm = c, g_rank = rank, g_world = world;
  return QNN_OK;
}

extern "C" int qnn_comm_destroy(void) {
  std::lock_guard<std::mutex> lock(g_comm_mu);
  if (!g_comm) return QNN_OK;
  const int rc = nccl_check(ncclCommDestroy(g_comm), "ncclCommDestroy");
  g_comm = nullptr, g_rank = -1, g_world = 0;
  return rc;
}

extern "C" int qnn_gather_f32(const float* send, float* recv, size_t count, int root, qnn_stream_t stream) {
  // held across the enqueue: a concurrent qnn_comm_destroy cannot free the communicator under it
  std::lock_guard<std::mutex> lock(g_comm_mu);
  QNN_REQUIRE(g_comm, "no communicator (qnn_comm_init)");
  QNN_REQUIRE(root >= 0 && root < g_world, "root out of range");
  if (count == 0) return QNN_OK;
  QNN_REQUIRE(send && (g_rank != root || recv), "null buffer");
  return nccl_check(ncclGather(send, recv, count, ncclFloat32, root, g_comm, (hipStream_t)stream), "ncclGather");
}
