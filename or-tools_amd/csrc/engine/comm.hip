// Multi-GPU collectives behind the C ABI: RCCL over xGMI.
//
// The batched configurations shard independent LPs across the GPUs of a node
// with no data-path collective; what crosses the GPUs is the search's bound,
// the cross-GPU analogue of SharedResponseManager::UpdateInnerObjectiveBounds
// (ortools/sat/synchronization.h:306): an all-reduce(min) (or max) of one
// float64. A C++ host (CP-SAT worker, MPSolver caller) reaches it through
// mi_lp_comm_* / mi_lp_share_bound without Python: one communicator per rank,
// its unique id passed out of band like ncclGetUniqueId's.
//
// RCCL is opened with dlopen(RTLD_LOCAL) from ROCm's librccl.so.1 and its
// entry points taken from that handle, so a process that also holds another
// RCCL copy (PyTorch's bundled librccl.so) never mixes the two: this one runs
// on the same HIP runtime as the engine's device buffers.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>

#include "../../../include/mi_lp.h"

namespace {

struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                             hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  std::string error;  // why the library is unusable, or empty
  bool ok() const { return error.empty(); }
};

const Rccl& Lib() {
  static Rccl* lib = [] {
    Rccl* r = new Rccl();  // process lifetime
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (h == nullptr) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (h == nullptr) {
      const char* e = dlerror();
      r->error = std::string("librccl.so.1: ") + (e ? e : "dlopen failed");
      return r;
    }
    auto sym = [&](const char* name) {
      void* p = dlsym(h, name);
      if (p == nullptr && r->error.empty()) r->error = std::string("librccl.so.1: no ") + name;
      return p;
    };
    r->get_unique_id = reinterpret_cast<decltype(r->get_unique_id)>(sym("ncclGetUniqueId"));
    r->comm_init_rank = reinterpret_cast<decltype(r->comm_init_rank)>(sym("ncclCommInitRank"));
    r->comm_destroy = reinterpret_cast<decltype(r->comm_destroy)>(sym("ncclCommDestroy"));
    r->all_reduce = reinterpret_cast<decltype(r->all_reduce)>(sym("ncclAllReduce"));
    r->all_gather = reinterpret_cast<decltype(r->all_gather)>(sym("ncclAllGather"));
    r->error_string = reinterpret_cast<decltype(r->error_string)>(sym("ncclGetErrorString"));
    return r;
  }();
  return *lib;
}

}  // namespace

struct mi_lp_comm {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  int32_t device = 0, rank = 0, nranks = 1;
  double* d_value = nullptr;  // the shared bound's device buffer (8 bytes)
  double* h_value = nullptr;  // pinned host mirror
  std::mutex mu;              // one collective at a time per communicator
  std::string error;
};

namespace {

int Fail(mi_lp_comm* c, const std::string& what) {
  if (c != nullptr) c->error = what;
  return MI_LP_ERROR_DEVICE;
}

int CheckHip(mi_lp_comm* c, hipError_t e, const char* what) {
  if (e == hipSuccess) return MI_LP_OK;
  return Fail(c, std::string(what) + ": " + hipGetErrorString(e));
}

int CheckNccl(mi_lp_comm* c, ncclResult_t e, const char* what) {
  if (e == ncclSuccess) return MI_LP_OK;
  return Fail(c, std::string(what) + ": " + Lib().error_string(e));
}

ncclRedOp_t RedOp(int32_t op) { return op == MI_LP_BOUND_MAX ? ncclMax : ncclMin; }

}  // namespace

extern "C" {

int mi_lp_comm_get_unique_id(uint8_t* id) {
  if (id == nullptr) return MI_LP_ERROR_NULL;
  const Rccl& r = Lib();
  if (!r.ok()) return MI_LP_ERROR_DEVICE;
  ncclUniqueId u;
  if (r.get_unique_id(&u) != ncclSuccess) return MI_LP_ERROR_DEVICE;
  static_assert(sizeof(u.internal) == MI_LP_COMM_ID_BYTES, "unique id size");
  std::memcpy(id, u.internal, MI_LP_COMM_ID_BYTES);
  return MI_LP_OK;
}

int mi_lp_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device,
                      mi_lp_comm** out) {
  if (id == nullptr || out == nullptr) return MI_LP_ERROR_NULL;
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks || device < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  const Rccl& r = Lib();
  if (!r.ok()) return MI_LP_ERROR_DEVICE;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device >= count) return MI_LP_ERROR_DEVICE;
  mi_lp_comm* c = new mi_lp_comm();
  c->device = device;
  c->rank = rank;
  c->nranks = nranks;
  int rc = CheckHip(c, hipSetDevice(device), "hipSetDevice");
  if (rc == MI_LP_OK) rc = CheckHip(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking),
                                    "hipStreamCreate");
  if (rc == MI_LP_OK) rc = CheckHip(c, hipMalloc(&c->d_value, sizeof(double)), "hipMalloc");
  if (rc == MI_LP_OK) {
    rc = CheckHip(c, hipHostMalloc(&c->h_value, sizeof(double), hipHostMallocDefault),
                  "hipHostMalloc");
  }
  if (rc == MI_LP_OK) {
    ncclUniqueId u;
    std::memcpy(u.internal, id, MI_LP_COMM_ID_BYTES);
    rc = CheckNccl(c, r.comm_init_rank(&c->comm, nranks, u, rank), "ncclCommInitRank");
  }
  if (rc != MI_LP_OK) {
    mi_lp_comm_destroy(c);
    return rc;
  }
  *out = c;
  return MI_LP_OK;
}

int32_t mi_lp_comm_rank(const mi_lp_comm* c) { return c == nullptr ? -1 : c->rank; }
int32_t mi_lp_comm_size(const mi_lp_comm* c) { return c == nullptr ? -1 : c->nranks; }

const char* mi_lp_comm_last_error(const mi_lp_comm* c) {
  if (c == nullptr) {
    const Rccl& r = Lib();
    return r.ok() ? "" : r.error.c_str();
  }
  return c->error.c_str();
}

int mi_lp_share_bound(mi_lp_comm* c, double* bound, int32_t op) {
  if (c == nullptr || bound == nullptr) return MI_LP_ERROR_NULL;
  if (op != MI_LP_BOUND_MIN && op != MI_LP_BOUND_MAX) return MI_LP_ERROR_INVALID_PROBLEM;
  std::lock_guard<std::mutex> lock(c->mu);
  int rc = CheckHip(c, hipSetDevice(c->device), "hipSetDevice");
  *c->h_value = *bound;
  if (rc == MI_LP_OK) {
    rc = CheckHip(c, hipMemcpyAsync(c->d_value, c->h_value, sizeof(double),
                                    hipMemcpyHostToDevice, c->stream), "bound H2D");
  }
  if (rc == MI_LP_OK) {
    rc = CheckNccl(c, Lib().all_reduce(c->d_value, c->d_value, 1, ncclFloat64, RedOp(op), c->comm,
                                       c->stream), "ncclAllReduce");
  }
  if (rc == MI_LP_OK) {
    rc = CheckHip(c, hipMemcpyAsync(c->h_value, c->d_value, sizeof(double),
                                    hipMemcpyDeviceToHost, c->stream), "bound D2H");
  }
  if (rc == MI_LP_OK) rc = CheckHip(c, hipStreamSynchronize(c->stream), "bound sync");
  if (rc == MI_LP_OK) *bound = *c->h_value;
  return rc;
}

int mi_lp_comm_allreduce_device(mi_lp_comm* c, double* d_values, int64_t count, int32_t op) {
  if (c == nullptr || (d_values == nullptr && count > 0)) return MI_LP_ERROR_NULL;
  if (count < 0 || (op != MI_LP_BOUND_MIN && op != MI_LP_BOUND_MAX)) {
    return MI_LP_ERROR_INVALID_PROBLEM;
  }
  if (count == 0) return MI_LP_OK;
  std::lock_guard<std::mutex> lock(c->mu);
  int rc = CheckHip(c, hipSetDevice(c->device), "hipSetDevice");
  if (rc == MI_LP_OK) {
    rc = CheckNccl(c, Lib().all_reduce(d_values, d_values, static_cast<size_t>(count), ncclFloat64,
                                       RedOp(op), c->comm, c->stream), "ncclAllReduce");
  }
  if (rc == MI_LP_OK) rc = CheckHip(c, hipStreamSynchronize(c->stream), "allreduce sync");
  return rc;
}

int mi_lp_comm_allgather_device(mi_lp_comm* c, const void* d_send, void* d_recv,
                                int64_t bytes_per_rank) {
  if (c == nullptr || ((d_send == nullptr || d_recv == nullptr) && bytes_per_rank > 0)) {
    return MI_LP_ERROR_NULL;
  }
  if (bytes_per_rank < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  if (bytes_per_rank == 0) return MI_LP_OK;
  std::lock_guard<std::mutex> lock(c->mu);
  int rc = CheckHip(c, hipSetDevice(c->device), "hipSetDevice");
  if (rc == MI_LP_OK) {
    rc = CheckNccl(c, Lib().all_gather(d_send, d_recv, static_cast<size_t>(bytes_per_rank),
                                       ncclUint8, c->comm, c->stream), "ncclAllGather");
  }
  if (rc == MI_LP_OK) rc = CheckHip(c, hipStreamSynchronize(c->stream), "allgather sync");
  return rc;
}

void mi_lp_comm_destroy(mi_lp_comm* c) {
  if (c == nullptr) return;
  (void)hipSetDevice(c->device);
  if (c->comm != nullptr) (void)Lib().comm_destroy(c->comm);
  if (c->stream != nullptr) (void)hipStreamDestroy(c->stream);
  if (c->d_value != nullptr) (void)hipFree(c->d_value);
  if (c->h_value != nullptr) (void)hipHostFree(c->h_value);
  delete c;
}

}  // extern "C"
