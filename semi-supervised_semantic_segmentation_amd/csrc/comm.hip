// Native RCCL communicator: the data-parallel gradient all-reduce and the SyncBN statistic sums of the training step
// (reference distributed_trainer.py:34-38: SyncBatchNorm conversion + DistributedDataParallel's bucketed reducer).
//
// Why the step does not use c10d's ProcessGroupNCCL: a captured HIP graph of a DDP step with c10d collectives breaks --
// c10d keeps a WorkNCCL per collective and its watchdog thread polls their events (hipEventQuery), which is refused
// while any stream of the process is capturing ("operation not permitted when stream is capturing"); in thread_local
// capture mode the poll passes, but the captured collectives' Work objects never complete outside a replay.  This
// communicator has no Work objects and no watchdog: an all-reduce is an RCCL enqueue on the caller's stream, which RCCL
// records into the graph being captured (persistent plan) like any kernel.
//
// RCCL is resolved at run time (dlopen) instead of linked: PyTorch-ROCm already has its own librccl loaded (soname
// librccl.so.1) when the process uses torch.distributed, and taking that copy (RTLD_NOLOAD first) keeps one RCCL in
// the process; a process without torch falls back to the system library.  libssseg.so itself therefore loads without
// RCCL (the ABI test runs on a CPU-only host).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "common.h"

namespace {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
};

RcclApi g_api;
std::once_flag g_once;
char g_err[256] = "";

template <typename F>
bool sym(void* h, const char* name, F& fn) {
  fn = reinterpret_cast<F>(dlsym(h, name));
  return fn != nullptr;
}

void load_api() {
  void* h = nullptr;
  // PyTorch's copy first (already mapped when torch.distributed is in use), then whatever the loader finds
  for (const char* n : {"librccl.so", "librccl.so.1"})
    if (!h) h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
  for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
    if (!h) h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    snprintf(g_err, sizeof(g_err), "ssseg comm: cannot load librccl (%s)", dlerror());
    return;
  }
  bool ok = sym(h, "ncclGetUniqueId", g_api.get_unique_id) && sym(h, "ncclCommInitRank", g_api.init_rank) &&
            sym(h, "ncclCommDestroy", g_api.destroy) && sym(h, "ncclAllReduce", g_api.all_reduce) &&
            sym(h, "ncclGroupStart", g_api.group_start) && sym(h, "ncclGroupEnd", g_api.group_end) &&
            sym(h, "ncclCommGetAsyncError", g_api.async_error) && sym(h, "ncclGetErrorString", g_api.error_string);
  if (!ok) {
    snprintf(g_err, sizeof(g_err), "ssseg comm: librccl lacks a required symbol");
    return;
  }
  g_api.ok = true;
}

bool api() {
  std::call_once(g_once, load_api);
  return g_api.ok;
}

// RCCL result -> ssseg return code: RCCL errors are reported as SSSEG_ECOMM with the message kept for
// ssseg_comm_last_error()
int rc(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return SSSEG_OK;
  snprintf(g_err, sizeof(g_err), "ssseg comm: %s: %s", what, g_api.error_string ? g_api.error_string(r) : "?");
  return SSSEG_ECOMM;
}

bool dtype_of(int dt, ncclDataType_t& out) {
  switch (dt) {
    case SSSEG_F32: out = ncclFloat32; return true;
    case SSSEG_BF16: out = ncclBfloat16; return true;
    case SSSEG_F16: out = ncclFloat16; return true;
    case SSSEG_F64: out = ncclFloat64; return true;
    default: return false;
  }
}

}  // namespace

extern "C" size_t ssseg_comm_unique_id_bytes(void) { return sizeof(ncclUniqueId); }

extern "C" const char* ssseg_comm_last_error(void) { return g_err; }

extern "C" int ssseg_comm_get_unique_id(void* uid_host) {
  if (!uid_host) return SSSEG_EINVAL;
  if (!api()) return SSSEG_ECOMM;
  ncclUniqueId id;
  const int r = rc(g_api.get_unique_id(&id), "ncclGetUniqueId");
  if (r == SSSEG_OK) memcpy(uid_host, &id, sizeof(id));
  return r;
}

extern "C" int ssseg_comm_init(ssseg_comm_t* comm_out, const void* uid_host, int rank, int world, int device) {
  if (!comm_out || !uid_host || world < 1 || rank < 0 || rank >= world || device < 0) return SSSEG_EINVAL;
  *comm_out = nullptr;
  if (!api()) return SSSEG_ECOMM;
  const hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) return (int)he;
  ncclUniqueId id;
  memcpy(&id, uid_host, sizeof(id));
  ncclComm_t c = nullptr;
  const int r = rc(g_api.init_rank(&c, world, id, rank), "ncclCommInitRank");
  if (r == SSSEG_OK) *comm_out = reinterpret_cast<ssseg_comm_t>(c);
  return r;
}

extern "C" int ssseg_comm_destroy(ssseg_comm_t comm) {
  if (!comm) return SSSEG_EINVAL;
  if (!api()) return SSSEG_ECOMM;
  return rc(g_api.destroy(reinterpret_cast<ncclComm_t>(comm)), "ncclCommDestroy");
}

extern "C" int ssseg_comm_async_error(ssseg_comm_t comm) {
  if (!comm) return SSSEG_EINVAL;
  if (!api()) return SSSEG_ECOMM;
  ncclResult_t e = ncclSuccess;
  const int r = rc(g_api.async_error(reinterpret_cast<ncclComm_t>(comm), &e), "ncclCommGetAsyncError");
  return r != SSSEG_OK ? r : rc(e, "asynchronous RCCL error");
}

// n in-place all-reduces fused into one RCCL group on `stream` (one kernel launch for the group).  op: SSSEG_SUM or
// SSSEG_AVG (RCCL's ncclAvg: the sum's one rounding, then the 1/world premultiplied scale -- the same arithmetic as
// c10d's ReduceOp.AVG on this backend, which is the same library call).
extern "C" int ssseg_allreduce_buckets(ssseg_comm_t comm, void* const* ptrs_host, const int64_t* counts_host, int64_t n,
                                       int dt, int op, ssseg_stream_t stream) {
  ncclDataType_t t;
  if (!comm || n < 0 || (n > 0 && (!ptrs_host || !counts_host)) || !dtype_of(dt, t)) return SSSEG_EINVAL;
  if (op != SSSEG_SUM && op != SSSEG_AVG) return SSSEG_EINVAL;
  for (int64_t i = 0; i < n; ++i)
    if (!ptrs_host[i] || counts_host[i] < 0) return SSSEG_EINVAL;
  if (n == 0) return SSSEG_OK;
  if (!api()) return SSSEG_ECOMM;
  const ncclRedOp_t o = op == SSSEG_AVG ? ncclAvg : ncclSum;
  ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
  if (n == 1) return rc(g_api.all_reduce(ptrs_host[0], ptrs_host[0], (size_t)counts_host[0], t, o, c, stream), "ncclAllReduce");
  int r = rc(g_api.group_start(), "ncclGroupStart");
  if (r != SSSEG_OK) return r;
  for (int64_t i = 0; i < n && r == SSSEG_OK; ++i)
    r = rc(g_api.all_reduce(ptrs_host[i], ptrs_host[i], (size_t)counts_host[i], t, o, c, stream), "ncclAllReduce");
  const int r2 = rc(g_api.group_end(), "ncclGroupEnd");
  return r != SSSEG_OK ? r : r2;
}
