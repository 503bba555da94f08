// RCCL over xGMI: one communicator per process/GPU.
// Replaces NCCL_Communicator (cuda/ntsCUDA.hpp:132-175; ncclCommInitAll +
// AllReduce/Bcast at cuda/ntsCUDAGraphOP.cu:173-193).  The reference runs one
// host thread per GPU inside a single process; here every GPU is its own
// process (torch.distributed launch), bootstrapped with a unique id that the
// host layer exchanges through the torch.distributed store.
#include <rccl/rccl.h>

#include "common.hpp"

struct nts_hip_comm {
  ncclComm_t comm = nullptr;
  int device = 0;
};

#define NTS_RCCL_TRY(expr)                                                               \
  do {                                                                                   \
    ncclResult_t _r = (expr);                                                            \
    if (_r != ncclSuccess) {                                                             \
      ::nts_hip::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,            \
                           ncclGetErrorString(_r));                                      \
      return NTS_ERR_RCCL;                                                               \
    }                                                                                    \
  } while (0)

static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId must be 128 bytes");

extern "C" {

int nts_hip_comm_unique_id(uint8_t out_id[128]) {
  NTS_CHECK_ARG(out_id, "out_id is NULL");
  ncclUniqueId id;
  NTS_RCCL_TRY(ncclGetUniqueId(&id));
  memcpy(out_id, &id, 128);
  return NTS_OK;
}

int nts_hip_comm_init(nts_hip_comm** out, int nranks, int rank, const uint8_t id[128],
                      int device) {
  NTS_CHECK_ARG(out && id, "NULL argument");
  NTS_CHECK_ARG(nranks > 0 && rank >= 0 && rank < nranks, "rank/nranks");
  *out = nullptr;
  NTS_HIP_TRY(hipSetDevice(device));
  ncclUniqueId uid;
  memcpy(&uid, id, 128);
  nts_hip_comm* c = new nts_hip_comm();
  c->device = device;
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    nts_hip::set_error("ncclCommInitRank failed: %s", ncclGetErrorString(r));
    delete c;
    return NTS_ERR_RCCL;
  }
  *out = c;
  return NTS_OK;
}

int nts_hip_comm_destroy(nts_hip_comm* c) {
  if (!c) return NTS_OK;
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
  return NTS_OK;
}

int nts_hip_comm_count(nts_hip_comm* c, int* nranks, int* rank) {
  NTS_CHECK_ARG(c && c->comm && nranks && rank, "NULL argument");
  NTS_RCCL_TRY(ncclCommCount(c->comm, nranks));
  NTS_RCCL_TRY(ncclCommUserRank(c->comm, rank));
  return NTS_OK;
}

int nts_hip_allreduce_sum_f32(nts_hip_comm* c, float* buf, uint64_t count, void* stream) {
  NTS_CHECK_ARG(c && c->comm && (buf || count == 0), "NULL argument");
  NTS_RCCL_TRY(ncclAllReduce(buf, buf, (size_t)count, ncclFloat, ncclSum, c->comm,
                             (hipStream_t)stream));
  return NTS_OK;
}

int nts_hip_broadcast_f32(nts_hip_comm* c, float* buf, uint64_t count, int root,
                          void* stream) {
  NTS_CHECK_ARG(c && c->comm && (buf || count == 0), "NULL argument");
  NTS_RCCL_TRY(ncclBroadcast(buf, buf, (size_t)count, ncclFloat, root, c->comm,
                             (hipStream_t)stream));
  return NTS_OK;
}

}  // extern "C"
