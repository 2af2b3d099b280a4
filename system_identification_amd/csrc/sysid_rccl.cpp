// sysid_rccl.cpp — the one exchange step of the multi-GPU path over RCCL:
// per-rank sysid_build_device / sysid_build_gram_device, then one in-place sum all-reduce of the
// (W+1)x(W+1) fp64 Gram over xGMI.  RCCL is resolved at run time (dlopen), preferring the copy already
// loaded in the process (PyTorch ships its own), so libsysid.so has no link-time dependency on it and
// a process never ends up with two RCCL instances.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>

#include "sysid.h"

namespace {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  std::string err;
};

thread_local std::string g_rccl_error;

Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* name : {"librccl.so.1", "librccl.so"}) {
      r.h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);  // already in the process (e.g. PyTorch's)
      if (r.h) break;
    }
    if (!r.h) r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!r.h) {
      r.err = std::string("cannot load librccl: ") + dlerror();
      return;
    }
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(r.h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(r.h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(r.h, "ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(r.h, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.h, "ncclGetErrorString"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.error_string) {
      r.err = "librccl lacks an expected symbol";
      r.h = nullptr;
    }
  });
  if (!r.h) {
    g_rccl_error = r.err;
    return nullptr;
  }
  return &r;
}

int fail(ncclResult_t st, Rccl* r, const char* what) {
  g_rccl_error = std::string(what) + ": " + (r ? r->error_string(st) : "rccl unavailable");
  return SYSID_E_DEVICE;
}

}  // namespace

extern "C" {

const char* sysid_rccl_last_error(void) { return g_rccl_error.c_str(); }

int32_t sysid_rccl_unique_id(void* id128) {
  if (!id128) return SYSID_E_INVALID;
  Rccl* r = rccl();
  if (!r) return SYSID_E_DEVICE;
  ncclUniqueId id;
  const ncclResult_t st = r->get_unique_id(&id);
  if (st != ncclSuccess) return fail(st, r, "ncclGetUniqueId");
  std::memcpy(id128, &id, sizeof(id));
  return SYSID_OK;
}

int32_t sysid_rccl_comm_init(void** comm, int32_t nranks, const void* id128, int32_t rank, int32_t device) {
  if (!comm || !id128 || nranks < 1 || rank < 0 || rank >= nranks) return SYSID_E_INVALID;
  Rccl* r = rccl();
  if (!r) return SYSID_E_DEVICE;
  if (hipSetDevice(device) != hipSuccess) {
    g_rccl_error = "hipSetDevice failed";
    return SYSID_E_DEVICE;
  }
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  ncclComm_t c = nullptr;
  const ncclResult_t st = r->comm_init_rank(&c, nranks, id, rank);
  if (st != ncclSuccess) return fail(st, r, "ncclCommInitRank");
  *comm = c;
  return SYSID_OK;
}

int32_t sysid_rccl_comm_destroy(void* comm) {
  if (!comm) return SYSID_OK;
  Rccl* r = rccl();
  if (!r) return SYSID_E_DEVICE;
  const ncclResult_t st = r->comm_destroy(static_cast<ncclComm_t>(comm));
  return st == ncclSuccess ? SYSID_OK : fail(st, r, "ncclCommDestroy");
}

int32_t sysid_allreduce_gram(const sysid_engine* e, double* d_gram, void* comm, void* stream) {
  if (!d_gram || !comm) return SYSID_E_INVALID;
  int32_t nq, nv, nj, nb, nc, cols, ld;
  if (sysid_dims(e, &nq, &nv, &nj, &nb, &nc, &cols, &ld) != SYSID_OK) return SYSID_E_INVALID;
  Rccl* r = rccl();
  if (!r) return SYSID_E_DEVICE;
  const ncclResult_t st = r->all_reduce(d_gram, d_gram, (size_t)cols * (size_t)cols, ncclFloat64, ncclSum,
                                        static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(stream));
  return st == ncclSuccess ? SYSID_OK : fail(st, r, "ncclAllReduce");
}

int32_t sysid_internal_xchg_pack(const sysid_engine* e, const double* d_gram, double rows, double* d_x, void* stream);
int32_t sysid_internal_xchg_unpack(const sysid_engine* e, const double* d_x, double* d_gram, void* stream);

int32_t sysid_allreduce_normal_equations(const sysid_engine* e, double* d_gram, double* d_xbuf, double rows,
                                         void* comm, void* stream) {
  if (!e || !d_gram || !d_xbuf || !comm || (reinterpret_cast<uintptr_t>(d_xbuf) & 7)) return SYSID_E_INVALID;
  Rccl* r = rccl();
  if (!r) return SYSID_E_DEVICE;
  const size_t count = sysid_exchange_bytes(e) / sizeof(double);
  if (sysid_internal_xchg_pack(e, d_gram, rows, d_xbuf, stream) != SYSID_OK) {
    g_rccl_error = "pack kernel launch failed";
    return SYSID_E_DEVICE;
  }
  const ncclResult_t st = r->all_reduce(d_xbuf, d_xbuf, count, ncclFloat64, ncclSum, static_cast<ncclComm_t>(comm),
                                        static_cast<hipStream_t>(stream));
  if (st != ncclSuccess) return fail(st, r, "ncclAllReduce");
  if (sysid_internal_xchg_unpack(e, d_xbuf, d_gram, stream) != SYSID_OK) {
    g_rccl_error = "unpack kernel launch failed";
    return SYSID_E_DEVICE;
  }
  return SYSID_OK;
}

}  // extern "C"
