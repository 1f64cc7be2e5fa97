// Native RCCL communicator: librccl driven directly from C++, not through
// torch.distributed's ProcessGroupNCCL.
//
// * The library is the RCCL torch already mapped (parallel/rccl.py passes the path of torch's bundled
//   librccl.so): dlopen returns the loaded copy, so there is one RCCL per process whichever side calls it.
// * Rendezvous: rank 0's ncclUniqueId travels through torch's TCPStore (env:// compatible, parallel/rccl.py);
//   every rank then calls ncclCommInitRank for its device.
// * Collectives are enqueued on a caller-chosen HIP stream and return at once: no Work objects, no event
//   bookkeeping - the caller orders them with stream waits (the gradient buckets go on a dedicated
//   high-priority comm stream behind the weight-gradient side stream, parallel/reducer.py).
// * Failure detection: ncclCommGetAsyncError is polled by the caller (peer death / network errors), and
//   ncclCommAbort tears a communicator down without waiting for peers.
//
// The RCCL header is included for its types only; every entry point is resolved with dlsym.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct Api {
  void* lib = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*get_version)(int*) = nullptr;
};

Api g_api;
std::mutex g_mu;
std::vector<ncclComm_t> g_comms;  // handle = index + 1; destroyed entries are null
std::string g_err;

template <typename F>
bool sym(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g_api.lib, name));
  if (!f) g_err = std::string("librccl: missing symbol ") + name;
  return f != nullptr;
}

ncclComm_t comm_of(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (h <= 0 || h > (int64_t)g_comms.size()) return nullptr;
  return g_comms[h - 1];
}

int fail(ncclResult_t r) {
  g_err = g_api.error_string ? g_api.error_string(r) : "rccl error";
  return (int)r;
}

}  // namespace

// 0 on success; the error text is rccl_last_error()
int rccl_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_api.lib) return 0;
  void* lib = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!lib) {
    g_err = std::string("dlopen ") + path + ": " + dlerror();
    return -1;
  }
  g_api.lib = lib;
  bool ok = sym(g_api.get_unique_id, "ncclGetUniqueId") && sym(g_api.comm_init_rank, "ncclCommInitRank") &&
            sym(g_api.all_reduce, "ncclAllReduce") && sym(g_api.broadcast, "ncclBroadcast") &&
            sym(g_api.comm_destroy, "ncclCommDestroy") && sym(g_api.comm_abort, "ncclCommAbort") &&
            sym(g_api.async_error, "ncclCommGetAsyncError") && sym(g_api.group_start, "ncclGroupStart") &&
            sym(g_api.group_end, "ncclGroupEnd") && sym(g_api.error_string, "ncclGetErrorString") &&
            sym(g_api.get_version, "ncclGetVersion");
  if (!ok) {
    g_api = Api{};
    return -1;
  }
  return 0;
}

const char* rccl_last_error() { return g_err.c_str(); }

int rccl_version() {
  int v = 0;
  if (!g_api.lib || g_api.get_version(&v) != ncclSuccess) return -1;
  return v;
}

int rccl_unique_id(char* out, int n) {
  if (!g_api.lib || n != NCCL_UNIQUE_ID_BYTES) return -1;
  ncclUniqueId id;
  const ncclResult_t r = g_api.get_unique_id(&id);
  if (r != ncclSuccess) return fail(r);
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

int rccl_comm_init(const char* uid, int n, int nranks, int rank, int device, int64_t* handle) {
  if (!g_api.lib || n != NCCL_UNIQUE_ID_BYTES) return -1;
  // ncclCommInitRank binds to the current device: select `device` for the call and restore the caller's
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
    g_err = "hipGetDevice / hipSetDevice failed";
    return -1;
  }
  ncclUniqueId id;
  std::memcpy(id.internal, uid, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t r = g_api.comm_init_rank(&c, nranks, id, rank);
  (void)hipSetDevice(prev);
  if (r != ncclSuccess) return fail(r);
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(c);
  *handle = (int64_t)g_comms.size();
  return 0;
}

// dtype: 0 fp32, 1 bf16, 2 fp64, 3 int32, 4 int64, 5 fp16; op: 0 sum, 1 max, 2 min, 3 prod
static bool map_types(int dtype, int op, ncclDataType_t* dt, ncclRedOp_t* ro) {
  switch (dtype) {
    case 0: *dt = ncclFloat32; break;
    case 1: *dt = ncclBfloat16; break;
    case 2: *dt = ncclFloat64; break;
    case 3: *dt = ncclInt32; break;
    case 4: *dt = ncclInt64; break;
    case 5: *dt = ncclFloat16; break;
    default: return false;
  }
  switch (op) {
    case 0: *ro = ncclSum; break;
    case 1: *ro = ncclMax; break;
    case 2: *ro = ncclMin; break;
    case 3: *ro = ncclProd; break;
    default: return false;
  }
  return true;
}

int rccl_all_reduce(int64_t h, void* buf, size_t count, int dtype, int op, hipStream_t stream) {
  ncclComm_t c = comm_of(h);
  ncclDataType_t dt;
  ncclRedOp_t ro;
  if (!c || !map_types(dtype, op, &dt, &ro)) {
    g_err = "rccl_all_reduce: bad handle / dtype / op";
    return -1;
  }
  const ncclResult_t r = g_api.all_reduce(buf, buf, count, dt, ro, c, stream);
  return r == ncclSuccess ? 0 : fail(r);
}

int rccl_broadcast(int64_t h, void* buf, size_t count, int dtype, int root, hipStream_t stream) {
  ncclComm_t c = comm_of(h);
  ncclDataType_t dt;
  ncclRedOp_t ro;
  if (!c || !map_types(dtype, 0, &dt, &ro)) {
    g_err = "rccl_broadcast: bad handle / dtype";
    return -1;
  }
  const ncclResult_t r = g_api.broadcast(buf, buf, count, dt, root, c, stream);
  return r == ncclSuccess ? 0 : fail(r);
}

int rccl_group(bool start) {
  if (!g_api.lib) return -1;
  const ncclResult_t r = start ? g_api.group_start() : g_api.group_end();
  return r == ncclSuccess ? 0 : fail(r);
}

// 0 = healthy, else the communicator's asynchronous error code (a dead peer, a network failure)
int rccl_async_error(int64_t h) {
  ncclComm_t c = comm_of(h);
  if (!c) return 0;  // closed or unknown handle: nothing left that could fail (teardown is not a fault)
  ncclResult_t e = ncclSuccess;
  const ncclResult_t r = g_api.async_error(c, &e);
  if (r != ncclSuccess) return fail(r);
  if (e != ncclSuccess && e != ncclInProgress) fail(e);
  return e == ncclInProgress ? 0 : (int)e;
}

int rccl_comm_close(int64_t h, bool abort) {
  ncclComm_t c = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (h <= 0 || h > (int64_t)g_comms.size() || !g_comms[h - 1]) return 0;
    c = g_comms[h - 1];
    g_comms[h - 1] = nullptr;
  }
  const ncclResult_t r = abort ? g_api.comm_abort(c) : g_api.comm_destroy(c);
  return r == ncclSuccess ? 0 : fail(r);
}
