// Native RCCL communicators (L4 of SURVEY.md §1): the MI355X replacement of
// the reference's MPI_Bcast / MPI_Send / MPI_Recv row traffic
// (OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:130-206), issued from C++
// on caller-chosen HIP streams.
//
// Why not only torch.distributed: ProcessGroupNCCL costs ~65 us of host time
// per collective (work objects, events, its watchdog), which at 8 ranks is
// more than a block step of the distributed solvers on the GPU
// (profiles/dist_issue_r5.md), and its watchdog thread queries the events of
// collectives recorded while a hipGraph is being captured, which aborts the
// process.  These communicators have none of that: one RCCL call per
// collective, graph-capturable, on the probed streams of utils/tensors.py.
//
// The library is the one torch already loaded (its path is passed in and
// dlopen returns the same handle), so there is exactly one RCCL in the
// process; no link-time dependency, libgelim loads without RCCL.  The unique
// id of each communicator is exchanged by the caller through the torch
// process group's store (parallel/comm.py).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>

#include "gelim/internal.h"

namespace {

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetVersion) version = nullptr;
};

Rccl g_rccl;
std::mutex g_rccl_mu;

int rccl_fail(ncclResult_t r, const char* what) {
  std::string msg = std::string(what) + ": " + (g_rccl.error_string ? g_rccl.error_string(r) : "RCCL error");
  return GELIM_FAIL(GELIM_E_HIP, msg);
}

#define RCCL_TRY(expr, what)                     \
  do {                                           \
    ncclResult_t _r = (expr);                    \
    if (_r != ncclSuccess) return rccl_fail(_r, what); \
  } while (0)

int need_loaded() {
  if (!g_rccl.handle) return GELIM_FAIL(GELIM_E_ARG, "RCCL not loaded (gelim_rccl_load)");
  return GELIM_OK;
}

bool dtype_of(int code, ncclDataType_t* t) {
  switch (code) {
    case 0: *t = ncclFloat64; return true;
    case 1: *t = ncclFloat32; return true;
    case 2: *t = ncclInt32; return true;
    case 3: *t = ncclInt64; return true;
    case 4: *t = ncclUint8; return true;
    default: return false;
  }
}

bool op_of(int code, ncclRedOp_t* op) {
  switch (code) {
    case 0: *op = ncclSum; return true;
    case 1: *op = ncclMax; return true;
    case 2: *op = ncclMin; return true;
    default: return false;
  }
}

}  // namespace

// dtype codes: 0 fp64, 1 fp32, 2 int32, 3 int64, 4 uint8; op codes: 0 sum, 1 max, 2 min.

// Bind the RCCL at `path` (torch's own librccl.so: already loaded, so the
// same instance).  Idempotent; 0 or an error code.
extern "C" int gelim_rccl_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (g_rccl.handle) return GELIM_OK;
  void* h = dlopen(path, RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
  if (!h) h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!h) return GELIM_FAIL(GELIM_E_IO, std::string("dlopen ") + path + ": " + dlerror());
  Rccl r;
  r.handle = h;
#define SYM(field, name)                                                                \
  r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, name));                        \
  if (!r.field) return GELIM_FAIL(GELIM_E_IO, std::string("RCCL symbol missing: ") + name);
  SYM(get_unique_id, "ncclGetUniqueId")
  SYM(init_rank, "ncclCommInitRank")
  SYM(destroy, "ncclCommDestroy")
  SYM(abort, "ncclCommAbort")
  SYM(async_error, "ncclCommGetAsyncError")
  SYM(error_string, "ncclGetErrorString")
  SYM(broadcast, "ncclBroadcast")
  SYM(all_reduce, "ncclAllReduce")
  SYM(all_gather, "ncclAllGather")
  SYM(send, "ncclSend")
  SYM(recv, "ncclRecv")
  SYM(group_start, "ncclGroupStart")
  SYM(group_end, "ncclGroupEnd")
  SYM(version, "ncclGetVersion")
#undef SYM
  g_rccl = r;
  return GELIM_OK;
}

extern "C" int gelim_rccl_version(void) {
  int v = 0;
  if (!g_rccl.handle || g_rccl.version(&v) != ncclSuccess) return -1;
  return v;
}

// 128 opaque bytes of a new communicator id (rank 0 of the communicator)
extern "C" int gelim_rccl_unique_id(uint8_t* out) {
  GELIM_TRY(need_loaded());
  ncclUniqueId id;
  RCCL_TRY(g_rccl.get_unique_id(&id), "ncclGetUniqueId");
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return GELIM_OK;
}

// Collective over the nranks callers with the same id, on the CURRENT HIP
// device.  *out = the communicator.
extern "C" int gelim_rccl_comm_create(void** out, const uint8_t* id_bytes, int32_t nranks, int32_t rank) {
  *out = nullptr;
  GELIM_TRY(need_loaded());
  if (nranks < 1 || rank < 0 || rank >= nranks) return GELIM_FAIL(GELIM_E_ARG, "rccl_comm_create: rank");
  ncclUniqueId id;
  std::memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  RCCL_TRY(g_rccl.init_rank(&c, nranks, id, rank), "ncclCommInitRank");
  *out = c;
  return GELIM_OK;
}

// abort = 1: ncclCommAbort (a peer failed; nothing pending is waited for)
extern "C" int gelim_rccl_comm_destroy(void* comm, int32_t abort) {
  if (!comm || !g_rccl.handle) return GELIM_OK;
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  RCCL_TRY(abort ? g_rccl.abort(c) : g_rccl.destroy(c), abort ? "ncclCommAbort" : "ncclCommDestroy");
  return GELIM_OK;
}

// 0 while healthy, else the GELIM error of the communicator's asynchronous
// failure (a dead peer, a network error): polled by the watchdog.
extern "C" int gelim_rccl_async_error(void* comm) {
  GELIM_TRY(need_loaded());
  ncclResult_t e = ncclSuccess;
  RCCL_TRY(g_rccl.async_error(static_cast<ncclComm_t>(comm), &e), "ncclCommGetAsyncError");
  if (e != ncclSuccess && e != ncclInProgress) return rccl_fail(e, "RCCL async error");
  return GELIM_OK;
}

// In place: buf on root is sent to every rank's buf.
extern "C" int gelim_rccl_bcast(void* comm, void* buf, int64_t count, int32_t dtype, int32_t root, void* stream) {
  GELIM_TRY(need_loaded());
  ncclDataType_t t;
  if (!dtype_of(dtype, &t) || count < 0) return GELIM_FAIL(GELIM_E_ARG, "rccl_bcast: dtype/count");
  RCCL_TRY(g_rccl.broadcast(buf, buf, (size_t)count, t, root, static_cast<ncclComm_t>(comm), (hipStream_t)stream),
           "ncclBroadcast");
  return GELIM_OK;
}

extern "C" int gelim_rccl_allreduce(void* comm, const void* send, void* recv, int64_t count, int32_t dtype,
                                    int32_t op, void* stream) {
  GELIM_TRY(need_loaded());
  ncclDataType_t t;
  ncclRedOp_t o;
  if (!dtype_of(dtype, &t) || !op_of(op, &o) || count < 0) return GELIM_FAIL(GELIM_E_ARG, "rccl_allreduce: args");
  RCCL_TRY(g_rccl.all_reduce(send, recv, (size_t)count, t, o, static_cast<ncclComm_t>(comm), (hipStream_t)stream),
           "ncclAllReduce");
  return GELIM_OK;
}

// recv holds nranks * count elements, rank order
extern "C" int gelim_rccl_allgather(void* comm, const void* send, void* recv, int64_t count, int32_t dtype,
                                    void* stream) {
  GELIM_TRY(need_loaded());
  ncclDataType_t t;
  if (!dtype_of(dtype, &t) || count < 0) return GELIM_FAIL(GELIM_E_ARG, "rccl_allgather: args");
  RCCL_TRY(g_rccl.all_gather(send, recv, (size_t)count, t, static_cast<ncclComm_t>(comm), (hipStream_t)stream),
           "ncclAllGather");
  return GELIM_OK;
}

// One grouped send to `dst` + receive from `src` (a ring step cannot deadlock
// on serialised send kernels); either side may be skipped with a null buffer.
extern "C" int gelim_rccl_sendrecv(void* comm, const void* send, int64_t scount, int32_t dst, void* recv,
                                   int64_t rcount, int32_t src, int32_t dtype, void* stream) {
  GELIM_TRY(need_loaded());
  ncclDataType_t t;
  if (!dtype_of(dtype, &t) || scount < 0 || rcount < 0) return GELIM_FAIL(GELIM_E_ARG, "rccl_sendrecv: args");
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  hipStream_t s = (hipStream_t)stream;
  RCCL_TRY(g_rccl.group_start(), "ncclGroupStart");
  ncclResult_t r1 = send ? g_rccl.send(send, (size_t)scount, t, dst, c, s) : ncclSuccess;
  ncclResult_t r2 = recv ? g_rccl.recv(recv, (size_t)rcount, t, src, c, s) : ncclSuccess;
  RCCL_TRY(g_rccl.group_end(), "ncclGroupEnd");
  if (r1 != ncclSuccess) return rccl_fail(r1, "ncclSend");
  if (r2 != ncclSuccess) return rccl_fail(r2, "ncclRecv");
  return GELIM_OK;
}
