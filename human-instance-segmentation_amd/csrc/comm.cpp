// RCCL communicator owned by libhiseg: the in-step collectives of data-parallel training (include/hiseg_comm.h).
// RCCL is resolved at run time from the library the process already loaded (torch's librccl.so), never linked,
// so one RCCL instance serves the process.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>
#include <mutex>
#include "hiseg.h"
#include "hiseg_comm.h"

void hiseg_set_error(const char* fmt, ...);

namespace {

struct Rccl {
  void* so = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl g_rccl;
std::mutex g_mu;

const char* rccl_err(ncclResult_t r) { return g_rccl.error_string ? g_rccl.error_string(r) : "?"; }

bool loaded(const char* what) {
  if (g_rccl.all_reduce) return true;
  hiseg_set_error("%s: RCCL not loaded (call hiseg_comm_load first)", what);
  return false;
}

}  // namespace

extern "C" int hiseg_comm_load(const char* path) {
  std::lock_guard<std::mutex> lock(g_mu);
  if (g_rccl.all_reduce) return HISEG_OK;
  const char* p = path ? path : "librccl.so";
  void* so = dlopen(p, RTLD_NOW | RTLD_GLOBAL);
  if (!so) {
    hiseg_set_error("comm_load: dlopen(%s): %s", p, dlerror());
    return HISEG_ERR_BAD_ARG;
  }
  Rccl r;
  r.so = so;
  r.get_unique_id = (decltype(r.get_unique_id))dlsym(so, "ncclGetUniqueId");
  r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(so, "ncclCommInitRank");
  r.all_reduce = (decltype(r.all_reduce))dlsym(so, "ncclAllReduce");
  r.comm_destroy = (decltype(r.comm_destroy))dlsym(so, "ncclCommDestroy");
  r.error_string = (decltype(r.error_string))dlsym(so, "ncclGetErrorString");
  if (!r.get_unique_id || !r.comm_init_rank || !r.all_reduce || !r.comm_destroy) {
    hiseg_set_error("comm_load: %s lacks an RCCL entry point", p);
    return HISEG_ERR_BAD_ARG;
  }
  g_rccl = r;
  return HISEG_OK;
}

extern "C" int hiseg_comm_unique_id(unsigned char* id_out) {
  if (!id_out) {
    hiseg_set_error("comm_unique_id: null output");
    return HISEG_ERR_BAD_ARG;
  }
  if (!loaded("comm_unique_id")) return HISEG_ERR_BAD_ARG;
  static_assert(sizeof(ncclUniqueId) == HISEG_COMM_ID_BYTES, "unique id size");
  ncclUniqueId id;
  const ncclResult_t r = g_rccl.get_unique_id(&id);
  if (r != ncclSuccess) {
    hiseg_set_error("comm_unique_id: %s", rccl_err(r));
    return HISEG_ERR_LAUNCH;
  }
  memcpy(id_out, id.internal, HISEG_COMM_ID_BYTES);
  return HISEG_OK;
}

extern "C" int hiseg_comm_init(hiseg_comm_t* comm, int nranks, const unsigned char* id, int rank, int device) {
  if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks || device < 0) {
    hiseg_set_error("comm_init: bad args (nranks %d rank %d device %d)", nranks, rank, device);
    return HISEG_ERR_BAD_ARG;
  }
  if (!loaded("comm_init")) return HISEG_ERR_BAD_ARG;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
    hiseg_set_error("comm_init: cannot select device %d", device);
    return HISEG_ERR_BAD_ARG;
  }
  ncclUniqueId uid;
  memcpy(uid.internal, id, HISEG_COMM_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t r = g_rccl.comm_init_rank(&c, nranks, uid, rank);
  (void)hipSetDevice(prev);
  if (r != ncclSuccess) {
    hiseg_set_error("comm_init: ncclCommInitRank(%d ranks, rank %d): %s", nranks, rank, rccl_err(r));
    return HISEG_ERR_LAUNCH;
  }
  *comm = (hiseg_comm_t)c;
  return HISEG_OK;
}

extern "C" int hiseg_comm_all_reduce(hiseg_comm_t comm, void* buf, long long count, int dtype, int op,
                                     hiseg_stream_t stream) {
  if (!comm || (!buf && count > 0) || count < 0 || (dtype != HISEG_COMM_F32 && dtype != HISEG_COMM_F64) ||
      (op != HISEG_COMM_SUM && op != HISEG_COMM_AVG)) {
    hiseg_set_error("comm_all_reduce: bad args (count %lld dtype %d op %d)", count, dtype, op);
    return HISEG_ERR_BAD_ARG;
  }
  if (!loaded("comm_all_reduce")) return HISEG_ERR_BAD_ARG;
  if (count == 0) return HISEG_OK;
  const ncclResult_t r =
      g_rccl.all_reduce(buf, buf, (size_t)count, dtype == HISEG_COMM_F32 ? ncclFloat32 : ncclFloat64,
                        op == HISEG_COMM_SUM ? ncclSum : ncclAvg, (ncclComm_t)comm, (hipStream_t)stream);
  if (r != ncclSuccess) {
    hiseg_set_error("comm_all_reduce: %s", rccl_err(r));
    return HISEG_ERR_LAUNCH;
  }
  return HISEG_OK;
}

extern "C" int hiseg_comm_destroy(hiseg_comm_t comm) {
  if (!comm) return HISEG_OK;
  if (!loaded("comm_destroy")) return HISEG_ERR_BAD_ARG;
  const ncclResult_t r = g_rccl.comm_destroy((ncclComm_t)comm);
  if (r != ncclSuccess) {
    hiseg_set_error("comm_destroy: %s", rccl_err(r));
    return HISEG_ERR_LAUNCH;
  }
  return HISEG_OK;
}
