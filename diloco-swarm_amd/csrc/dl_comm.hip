// RCCL entry points of the C-ABI (dl_allreduce(buf, count, dtype, comm,
// stream)) for hosts that drive the exchange themselves instead of through torch.distributed.
//
// RCCL is resolved at run time, not linked: a communicator must be used with the RCCL that
// created it, and a PyTorch process already carries its own copy (the one behind
// ProcessGroupNCCL, whose ncclComm_t `_comm_ptr()` returns). dl_rccl_load(path) picks the
// library; with NULL it takes the RCCL already loaded in the process, else librccl.so.1.
// Each collective is enqueued on the caller's stream, SUM, in place where the RCCL API allows.
#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <mutex>

#include <rccl/rccl.h>

#include "dl_internal.h"

namespace {

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclGetVersion) get_version = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
};

std::mutex g_mu;
Rccl g_rccl;

int err(int code, const char* fmt, const char* a = "", const char* b = "") {
  char buf[512];
  std::snprintf(buf, sizeof buf, fmt, a, b);
  return dl::set_error(code, buf);
}

template <class F>
bool sym(void* h, const char* name, F* out) {
  *out = reinterpret_cast<F>(dlsym(h, name));
  return *out != nullptr;
}

int bind(void* h, const char* what) {
  Rccl r;
  r.handle = h;
  if (!sym(h, "ncclGetUniqueId", &r.get_unique_id) ||
      !sym(h, "ncclCommInitRank", &r.comm_init_rank) ||
      !sym(h, "ncclCommDestroy", &r.comm_destroy) || !sym(h, "ncclAllReduce", &r.all_reduce) ||
      !sym(h, "ncclReduceScatter", &r.reduce_scatter) ||
      !sym(h, "ncclAllGather", &r.all_gather) ||
      !sym(h, "ncclGetErrorString", &r.error_string) ||
      !sym(h, "ncclGetVersion", &r.get_version) || !sym(h, "ncclSend", &r.send) ||
      !sym(h, "ncclRecv", &r.recv) || !sym(h, "ncclGroupStart", &r.group_start) ||
      !sym(h, "ncclGroupEnd", &r.group_end))
    return err(DL_E_STATE, "dl_rccl_load: %s lacks an RCCL entry point", what);
  g_rccl = r;
  return DL_OK;
}

int load_locked(const char* path) {
  if (path && *path) {
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) return err(DL_E_STATE, "dl_rccl_load: cannot open %s (%s)", path, dlerror());
    return bind(h, path);
  }
  // the RCCL already in the process (torch's), then the ROCm one
  const char* loaded[] = {"librccl.so", "librccl.so.1"};
  for (const char* n : loaded)
    if (void* h = dlopen(n, RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD)) return bind(h, n);
  const char* fresh[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
  for (const char* n : fresh)
    if (void* h = dlopen(n, RTLD_NOW | RTLD_LOCAL)) return bind(h, n);
  return err(DL_E_STATE, "dl_rccl_load: no RCCL library found%s%s");
}

int ready(const char* who) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_rccl.handle) return DL_OK;
  int rc = load_locked(nullptr);
  if (rc) return rc;
  (void)who;
  return DL_OK;
}

int rccl_fail(ncclResult_t r, const char* who) {
  return err(DL_E_RCCL, "%s: %s", who, g_rccl.error_string ? g_rccl.error_string(r) : "?");
}

bool dtype_of(int32_t dt, ncclDataType_t* out, size_t* bytes) {
  switch (dt) {
    case DL_F32: *out = ncclFloat32; *bytes = 4; return true;
    case DL_BF16: *out = ncclBfloat16; *bytes = 2; return true;
    case DL_F16: *out = ncclFloat16; *bytes = 2; return true;
    case DL_U8: *out = ncclUint8; *bytes = 1; return true;
    default: return false;
  }
}

#define DL_RCCL_ARGS(who, comm, dt)                                               \
  do {                                                                            \
    if (int rc_ = ready(who)) return rc_;                                         \
    if (!(comm)) return err(DL_E_ARG, "%s: null communicator", who);              \
    if (!dtype_of(dt, &nt, &eb)) return err(DL_E_ARG, "%s: unsupported dtype", who); \
  } while (0)

}  // namespace

extern "C" {

DL_API int dl_rccl_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_mu);
  return load_locked(path);
}

DL_API int dl_rccl_version(int32_t* version) {
  if (int rc = ready("dl_rccl_version")) return rc;
  if (!version) return err(DL_E_ARG, "dl_rccl_version: null argument");
  int v = 0;
  ncclResult_t r = g_rccl.get_version(&v);
  if (r != ncclSuccess) return rccl_fail(r, "dl_rccl_version");
  *version = v;
  return DL_OK;
}

DL_API int dl_comm_unique_id(void* id) {
  if (int rc = ready("dl_comm_unique_id")) return rc;
  if (!id) return err(DL_E_ARG, "dl_comm_unique_id: null id");
  ncclResult_t r = g_rccl.get_unique_id(static_cast<ncclUniqueId*>(id));
  return r == ncclSuccess ? DL_OK : rccl_fail(r, "dl_comm_unique_id");
}

DL_API int dl_comm_init(dl_comm_t* out, int32_t nranks, const void* id, int32_t rank) {
  if (int rc = ready("dl_comm_init")) return rc;
  if (!out || !id) return err(DL_E_ARG, "dl_comm_init: null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return err(DL_E_ARG, "dl_comm_init: bad rank / nranks");
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  ncclComm_t c = nullptr;
  ncclResult_t r = g_rccl.comm_init_rank(&c, nranks, uid, rank);
  if (r != ncclSuccess) return rccl_fail(r, "dl_comm_init");
  *out = c;
  return DL_OK;
}

DL_API int dl_comm_destroy(dl_comm_t comm) {
  if (!comm) return DL_OK;
  if (int rc = ready("dl_comm_destroy")) return rc;
  ncclResult_t r = g_rccl.comm_destroy(static_cast<ncclComm_t>(comm));
  return r == ncclSuccess ? DL_OK : rccl_fail(r, "dl_comm_destroy");
}

DL_API int dl_allreduce(void* buf, int64_t count, int32_t dtype, dl_comm_t comm, dl_stream_t s) {
  ncclDataType_t nt;
  size_t eb;
  DL_RCCL_ARGS("dl_allreduce", comm, dtype);
  if (count < 0 || (count > 0 && !buf)) return err(DL_E_ARG, "dl_allreduce: bad buffer");
  if (count == 0) return DL_OK;
  ncclResult_t r = g_rccl.all_reduce(buf, buf, size_t(count), nt, ncclSum,
                                     static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(s));
  return r == ncclSuccess ? DL_OK : rccl_fail(r, "dl_allreduce");
}

DL_API int dl_reduce_scatter(const void* send, void* recv, int64_t recv_count, int32_t dtype,
                             dl_comm_t comm, dl_stream_t s) {
  ncclDataType_t nt;
  size_t eb;
  DL_RCCL_ARGS("dl_reduce_scatter", comm, dtype);
  if (recv_count < 0 || (recv_count > 0 && (!send || !recv)))
    return err(DL_E_ARG, "dl_reduce_scatter: bad buffer");
  if (recv_count == 0) return DL_OK;
  ncclResult_t r = g_rccl.reduce_scatter(send, recv, size_t(recv_count), nt, ncclSum,
                                         static_cast<ncclComm_t>(comm),
                                         static_cast<hipStream_t>(s));
  return r == ncclSuccess ? DL_OK : rccl_fail(r, "dl_reduce_scatter");
}

DL_API int dl_all_gather(const void* send, void* recv, int64_t send_count, int32_t dtype,
                         dl_comm_t comm, dl_stream_t s) {
  ncclDataType_t nt;
  size_t eb;
  DL_RCCL_ARGS("dl_all_gather", comm, dtype);
  if (send_count < 0 || (send_count > 0 && (!send || !recv)))
    return err(DL_E_ARG, "dl_all_gather: bad buffer");
  if (send_count == 0) return DL_OK;
  ncclResult_t r = g_rccl.all_gather(send, recv, size_t(send_count), nt,
                                     static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(s));
  return r == ncclSuccess ? DL_OK : rccl_fail(r, "dl_all_gather");
}

/* Point-to-point (the payload leg of the device pipeline transport,
 * replacing the reference's dist.send / dist.recv of a host copy, src/comm.py:38,67).
 * Calls between dl_group_start and dl_group_end are issued as one RCCL group (a send and
 * its matching receive on one rank -- a self send -- must be grouped). */
DL_API int dl_send(const void* buf, int64_t count, int32_t dtype, int32_t peer, dl_comm_t comm,
                   dl_stream_t s) {
  ncclDataType_t nt;
  size_t eb;
  DL_RCCL_ARGS("dl_send", comm, dtype);
  if (count < 0 || (count > 0 && !buf) || peer < 0) return err(DL_E_ARG, "dl_send: bad argument");
  ncclResult_t r = g_rccl.send(buf, size_t(count), nt, peer, static_cast<ncclComm_t>(comm),
                               static_cast<hipStream_t>(s));
  return r == ncclSuccess ? DL_OK : rccl_fail(r, "dl_send");
}

DL_API int dl_recv(void* buf, int64_t count, int32_t dtype, int32_t peer, dl_comm_t comm,
                   dl_stream_t s) {
  ncclDataType_t nt;
  size_t eb;
  DL_RCCL_ARGS("dl_recv", comm, dtype);
  if (count < 0 || (count > 0 && !buf) || peer < 0) return err(DL_E_ARG, "dl_recv: bad argument");
  ncclResult_t r = g_rccl.recv(buf, size_t(count), nt, peer, static_cast<ncclComm_t>(comm),
                               static_cast<hipStream_t>(s));
  return r == ncclSuccess ? DL_OK : rccl_fail(r, "dl_recv");
}

DL_API int dl_group_start(void) {
  if (int rc = ready("dl_group_start")) return rc;
  ncclResult_t r = g_rccl.group_start();
  return r == ncclSuccess ? DL_OK : rccl_fail(r, "dl_group_start");
}

DL_API int dl_group_end(void) {
  if (int rc = ready("dl_group_end")) return rc;
  ncclResult_t r = g_rccl.group_end();
  return r == ncclSuccess ? DL_OK : rccl_fail(r, "dl_group_end");
}

}  // extern "C"
