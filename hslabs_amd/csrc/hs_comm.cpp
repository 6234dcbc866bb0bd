// hs_comm.cpp -- the path's single collective: the best-rollout reduce across the ranks of a
// job, one process per GPU, as one RCCL all-reduce(MIN) of the 8-byte key (ncclUint64) over
// xGMI. The reference has no counterpart (it sweeps serially in one process,
// player.cpp:311-321); rollouts are sharded in contiguous id ranges, so the reduced key names
// the global winner. The message is 8 bytes: latency-bound, one call per job.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "hs_internal.h"

static_assert(HS_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "hs_comm id size is RCCL's unique id size");

struct hs_comm_s {
  ncclComm_t comm = nullptr;
  int dev = 0;
  int32_t n_ranks = 0, rank = 0;
  uint64_t* scratch = nullptr;  // 8 B on dev: hs_select_best_comm's reduce buffer (never a batch's own key)
};

namespace {

int nccl_fail(ncclResult_t r, const char* what) {
  return hs::set_error(HS_E_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}

}  // namespace

namespace hs {

int comm_reduce_min(hs_comm_t c, uint64_t* key, void* stream) {
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e != hipSuccess) return set_error(HS_E_DEVICE, std::string("hipGetDevice: ") + hipGetErrorString(e));
  if (cur != c->dev && (e = hipSetDevice(c->dev)) != hipSuccess)
    return set_error(HS_E_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
  ncclResult_t r = ncclAllReduce(key, key, 1, ncclUint64, ncclMin, c->comm, (hipStream_t)stream);
  if (cur != c->dev) (void)hipSetDevice(cur);
  if (r != ncclSuccess) return nccl_fail(r, "ncclAllReduce(best key)");
  return HS_OK;
}

int comm_device(hs_comm_t c) { return c->dev; }

uint64_t* comm_scratch(hs_comm_t c) { return c->scratch; }

}  // namespace hs

extern "C" {

int hs_comm_unique_id(char id[HS_COMM_ID_BYTES]) {
  if (!id) return hs::set_error(HS_E_ARG, "null id");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
  std::memcpy(id, u.internal, HS_COMM_ID_BYTES);
  return HS_OK;
}

int hs_comm_init(int32_t n_ranks, int32_t rank, const char id[HS_COMM_ID_BYTES], hs_comm_t* out) {
  if (!id || !out) return hs::set_error(HS_E_ARG, "null argument");
  *out = nullptr;
  if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return hs::set_error(HS_E_ARG, "rank out of [0, n_ranks)");
  auto* c = new hs_comm_s;
  hipError_t e = hipGetDevice(&c->dev);
  if (e != hipSuccess) {
    delete c;
    return hs::set_error(HS_E_DEVICE, std::string("hipGetDevice: ") + hipGetErrorString(e));
  }
  ncclUniqueId u;
  std::memcpy(u.internal, id, HS_COMM_ID_BYTES);
  ncclResult_t r = ncclCommInitRank(&c->comm, n_ranks, u, rank);  // collective over the ranks
  if (r != ncclSuccess) {
    delete c;
    return nccl_fail(r, "ncclCommInitRank");
  }
  c->n_ranks = n_ranks;
  c->rank = rank;
  e = hipMalloc(&c->scratch, sizeof(uint64_t));
  if (e != hipSuccess) {
    (void)ncclCommDestroy(c->comm);
    delete c;
    return hs::set_error(HS_E_DEVICE, std::string("hipMalloc(comm scratch): ") + hipGetErrorString(e));
  }
  *out = c;
  return HS_OK;
}

void hs_comm_free(hs_comm_t c) {
  if (!c) return;
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->scratch) {
    int cur = 0;
    if (hipGetDevice(&cur) == hipSuccess && hipSetDevice(c->dev) == hipSuccess) {
      (void)hipFree(c->scratch);
      (void)hipSetDevice(cur);
    }
  }
  delete c;
}

int hs_comm_size(hs_comm_t c, int32_t* n_ranks, int32_t* rank) {
  if (!c) return hs::set_error(HS_E_ARG, "null comm");
  if (n_ranks) *n_ranks = c->n_ranks;
  if (rank) *rank = c->rank;
  return HS_OK;
}

int hs_comm_reduce_best(hs_comm_t c, uint64_t* key, void* stream) {
  if (!c || !key) return hs::set_error(HS_E_ARG, "null comm or key");
  return hs::comm_reduce_min(c, key, stream);
}

}  // extern "C"
