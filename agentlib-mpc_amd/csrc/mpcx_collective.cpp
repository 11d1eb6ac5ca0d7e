// mpcx_collective.cpp — the one collective of an ADMM iteration, issued by the library (C ABI v14).
//
// the library owns the per-iteration all-reduce of the ADMM fleet (the sum of the
// global groups' moments, the rank-spanning blocks' residual totals and the control double,
// mpcx_admm_reduce_count doubles) instead of leaving it to the caller.  The reference has no
// counterpart on one process (its agents exchange JSON messages through a broker); the exchange
// this replaces is the coordinator's gather of every agent's locals and its broadcast of the means
// (modules/dmpc/admm/admm_coordinator.py:284-314) when the agents sit on several GPUs.
//
// Two transports, registered once per process (one process per GPU):
//   * RCCL: a communicator (ncclComm_t) and the RCCL library that made it.  RCCL is resolved at
//     registration with dlopen / dlsym, not linked: a Python process already holds PyTorch's own
//     librccl (its communicators come from that copy), a C caller the system's.  The library then
//     calls ncclAllReduce(sum, fp64, in place) on the caller's HIP stream.  mpcx_rccl_comm_init /
//     mpcx_rccl_comm_init_file create such a communicator (the latter with a shared-file bootstrap
//     of the unique id, so a C caller needs no other collective library).
//   * a function: any other transport (gloo through PyTorch on the CPU, MPI, a test stub).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>

#include "mpcx.h"

namespace {

typedef ncclResult_t (*fn_get_unique_id)(ncclUniqueId*);
typedef ncclResult_t (*fn_comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
typedef ncclResult_t (*fn_comm_destroy)(ncclComm_t);
typedef ncclResult_t (*fn_all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                      hipStream_t);
typedef const char* (*fn_error_string)(ncclResult_t);

struct Rccl {
  void* dl = nullptr;
  fn_get_unique_id get_unique_id = nullptr;
  fn_comm_init_rank comm_init_rank = nullptr;
  fn_comm_destroy comm_destroy = nullptr;
  fn_all_reduce all_reduce = nullptr;
  fn_error_string error_string = nullptr;
};

// an RCCL copy already in the process (RTLD_NOLOAD) is preferred: communicators must be used
// with the library instance that created them
int open_rccl(const char* path, Rccl* r) {
  const char* p = (path != nullptr && path[0] != '\0') ? path : "librccl.so.1";
  void* dl = dlopen(p, RTLD_NOW | RTLD_NOLOAD);
  if (dl == nullptr) dl = dlopen(p, RTLD_NOW | RTLD_LOCAL);
  if (dl == nullptr) {
    std::fprintf(stderr, "mpcx: cannot load RCCL (%s): %s\n", p, dlerror());
    return MPCX_ERR_COMM;
  }
  Rccl out;
  out.dl = dl;
  out.get_unique_id = (fn_get_unique_id)dlsym(dl, "ncclGetUniqueId");
  out.comm_init_rank = (fn_comm_init_rank)dlsym(dl, "ncclCommInitRank");
  out.comm_destroy = (fn_comm_destroy)dlsym(dl, "ncclCommDestroy");
  out.all_reduce = (fn_all_reduce)dlsym(dl, "ncclAllReduce");
  out.error_string = (fn_error_string)dlsym(dl, "ncclGetErrorString");
  if (!out.get_unique_id || !out.comm_init_rank || !out.comm_destroy || !out.all_reduce) {
    std::fprintf(stderr, "mpcx: %s lacks the RCCL entry points\n", p);
    dlclose(dl);
    return MPCX_ERR_COMM;
  }
  *r = out;
  return MPCX_OK;
}

int rccl_fail(const Rccl& r, ncclResult_t e, const char* what) {
  std::fprintf(stderr, "mpcx: %s failed: %s\n", what, r.error_string ? r.error_string(e) : "RCCL error");
  return MPCX_ERR_COMM;
}

// the registered transport (process-wide)
std::mutex g_mu;
int g_kind = MPCX_COLLECTIVE_NONE;
Rccl g_rccl;
ncclComm_t g_comm = nullptr;
mpcx_allreduce_fn g_fn = nullptr;
void* g_ctx = nullptr;
std::atomic<long long> g_calls{0};

}  // namespace

extern "C" int mpcx_allreduce_register(void* comm, const char* rccl_library) {
  if (comm == nullptr) return MPCX_ERR_ARG;
  Rccl r;
  const int rc = open_rccl(rccl_library, &r);
  if (rc != MPCX_OK) return rc;
  std::lock_guard<std::mutex> lk(g_mu);
  g_rccl = r;
  g_comm = (ncclComm_t)comm;
  g_fn = nullptr;
  g_ctx = nullptr;
  g_kind = MPCX_COLLECTIVE_RCCL;
  return MPCX_OK;
}

extern "C" int mpcx_allreduce_register_fn(mpcx_allreduce_fn fn, void* ctx) {
  if (fn == nullptr) return MPCX_ERR_ARG;
  std::lock_guard<std::mutex> lk(g_mu);
  g_fn = fn;
  g_ctx = ctx;
  g_comm = nullptr;
  g_kind = MPCX_COLLECTIVE_FN;
  return MPCX_OK;
}

extern "C" int mpcx_allreduce_unregister(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_kind = MPCX_COLLECTIVE_NONE;
  g_comm = nullptr;
  g_fn = nullptr;
  g_ctx = nullptr;
  return MPCX_OK;
}

extern "C" int mpcx_allreduce_kind(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_kind;
}

extern "C" int64_t mpcx_allreduce_calls(void) { return (int64_t)g_calls.load(); }

extern "C" int mpcx_admm_allreduce(double* buf, int64_t count, void* stream) {
  if (count < 0 || (count > 0 && buf == nullptr)) return MPCX_ERR_ARG;
  int kind;
  Rccl r;
  ncclComm_t comm;
  mpcx_allreduce_fn fn;
  void* ctx;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    kind = g_kind; r = g_rccl; comm = g_comm; fn = g_fn; ctx = g_ctx;
  }
  if (kind == MPCX_COLLECTIVE_NONE) return MPCX_ERR_COMM;
  g_calls.fetch_add(1);
  if (kind == MPCX_COLLECTIVE_FN) return fn(ctx, buf, count, stream) == 0 ? MPCX_OK : MPCX_ERR_COMM;
  const ncclResult_t e = r.all_reduce(buf, buf, (size_t)count, ncclFloat64, ncclSum, comm, (hipStream_t)stream);
  return e == ncclSuccess ? MPCX_OK : rccl_fail(r, e, "ncclAllReduce");
}

extern "C" int mpcx_rccl_unique_id(const char* rccl_library, void* id) {
  if (id == nullptr) return MPCX_ERR_ARG;
  Rccl r;
  const int rc = open_rccl(rccl_library, &r);
  if (rc != MPCX_OK) return rc;
  ncclUniqueId u;
  const ncclResult_t e = r.get_unique_id(&u);
  if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
  std::memcpy(id, &u, sizeof(u));
  return MPCX_OK;
}

extern "C" int mpcx_rccl_comm_init(const char* rccl_library, int32_t nranks, int32_t rank, const void* id,
                                   void** comm) {
  if (comm == nullptr || id == nullptr || nranks < 1 || rank < 0 || rank >= nranks) return MPCX_ERR_ARG;
  *comm = nullptr;
  Rccl r;
  const int rc = open_rccl(rccl_library, &r);
  if (rc != MPCX_OK) return rc;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  const ncclResult_t e = r.comm_init_rank(&c, nranks, u, rank);
  if (e != ncclSuccess) return rccl_fail(r, e, "ncclCommInitRank");
  *comm = (void*)c;
  return MPCX_OK;
}

extern "C" int mpcx_rccl_comm_init_file(const char* rccl_library, const char* id_path, int32_t nranks,
                                        int32_t rank, int32_t timeout_ms, void** comm) {
  if (id_path == nullptr || comm == nullptr || nranks < 1 || rank < 0 || rank >= nranks) return MPCX_ERR_ARG;
  unsigned char id[MPCX_RCCL_ID_BYTES];
  if (rank == 0) {
    int rc = mpcx_rccl_unique_id(rccl_library, id);
    if (rc != MPCX_OK) return rc;
    // written beside, then renamed: a reader sees the whole id or nothing
    const std::string tmp = std::string(id_path) + ".tmp." + std::to_string((long)getpid());
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (f == nullptr) return MPCX_ERR_COMM;
    const size_t nw = std::fwrite(id, 1, sizeof(id), f);
    std::fclose(f);
    if (nw != sizeof(id) || std::rename(tmp.c_str(), id_path) != 0) return MPCX_ERR_COMM;
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      FILE* f = std::fopen(id_path, "rb");
      if (f != nullptr) {
        const size_t nr = std::fread(id, 1, sizeof(id), f);
        std::fclose(f);
        if (nr == sizeof(id)) break;
      }
      const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0);
      if (ms.count() > timeout_ms) return MPCX_ERR_COMM;
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
  }
  return mpcx_rccl_comm_init(rccl_library, nranks, rank, id, comm);
}

extern "C" int mpcx_rccl_comm_destroy(const char* rccl_library, void* comm) {
  if (comm == nullptr) return MPCX_ERR_ARG;
  Rccl r;
  const int rc = open_rccl(rccl_library, &r);
  if (rc != MPCX_OK) return rc;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_kind == MPCX_COLLECTIVE_RCCL && g_comm == (ncclComm_t)comm) {
      g_kind = MPCX_COLLECTIVE_NONE;
      g_comm = nullptr;
    }
  }
  const ncclResult_t e = r.comm_destroy((ncclComm_t)comm);
  return e == ncclSuccess ? MPCX_OK : rccl_fail(r, e, "ncclCommDestroy");
}
