// Native RCCL communicator for the data-parallel step (xGMI all-reduce issued from C++).
//
// torch.distributed's ProcessGroupNCCL runs every collective on its own internal stream behind
// event hand-offs and a Python call (tens of microseconds of host time per collective); the
// step's collectives are few, large and at fixed points, so the engine drives RCCL directly:
// ncclAllReduce on the engine's comm stream, ordered against the compute streams by the same
// events the schedule already uses, and capturable into a hipGraph.
//
// The library is the RCCL that PyTorch itself loaded (its bundled librccl.so, path given by the
// caller), resolved with dlopen / dlsym: one RCCL per process, no link-time dependency, and the
// communicator is our own (created from a unique id that rank 0 makes and the process group
// broadcasts), so it never shares queues or state with torch's.
#pragma once
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdexcept>
#include <string>

namespace dcg_comm {

struct Rccl {
  void* lib = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;

  void load(const std::string& path) {
    if (lib) return;
    lib = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!lib) throw std::runtime_error("RCCL: dlopen(" + path + ") failed: " + std::string(dlerror()));
    auto sym = [&](const char* n) {
      void* p = dlsym(lib, n);
      if (!p) throw std::runtime_error(std::string("RCCL: missing symbol ") + n);
      return p;
    };
    get_unique_id = reinterpret_cast<decltype(get_unique_id)>(sym("ncclGetUniqueId"));
    comm_init_rank = reinterpret_cast<decltype(comm_init_rank)>(sym("ncclCommInitRank"));
    all_reduce = reinterpret_cast<decltype(all_reduce)>(sym("ncclAllReduce"));
    comm_destroy = reinterpret_cast<decltype(comm_destroy)>(sym("ncclCommDestroy"));
    error_string = reinterpret_cast<decltype(error_string)>(sym("ncclGetErrorString"));
  }
  void check(ncclResult_t r, const char* what) const {
    if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + error_string(r));
  }
};

inline Rccl& rccl() {
  static Rccl r;
  return r;
}

// dtype codes of the Python side: 0 = fp32, 1 = bf16, 2 = fp16
inline ncclDataType_t nccl_type(int code) {
  switch (code) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    default: throw std::runtime_error("RCCL: bad dtype code " + std::to_string(code));
  }
}

class Comm {
 public:
  // a fresh unique id (rank 0), as 128 raw bytes
  static std::string unique_id(const std::string& lib_path) {
    rccl().load(lib_path);
    ncclUniqueId id;
    rccl().check(rccl().get_unique_id(&id), "ncclGetUniqueId");
    return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
  }

  Comm(const std::string& lib_path, int nranks, int rank, const std::string& id_bytes, int device)
      : nranks_(nranks), rank_(rank) {
    if ((int)id_bytes.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("RCCL: unique id must be 128 bytes");
    rccl().load(lib_path);
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("RCCL: hipSetDevice failed");
    ncclUniqueId id;
    std::copy(id_bytes.begin(), id_bytes.end(), id.internal);
    rccl().check(rccl().comm_init_rank(&comm_, nranks, id, rank), "ncclCommInitRank");
  }
  ~Comm() { destroy(); }

  void destroy() {
    if (comm_) {
      rccl().comm_destroy(comm_);
      comm_ = nullptr;
    }
  }

  // in-place SUM all-reduce of count elements at ptr, enqueued on `stream` (a hipStream_t)
  void all_reduce(uintptr_t ptr, size_t count, int dtype, uintptr_t stream) {
    if (!comm_) throw std::runtime_error("RCCL: communicator destroyed");
    void* p = reinterpret_cast<void*>(ptr);
    rccl().check(rccl().all_reduce(p, p, count, nccl_type(dtype), ncclSum, comm_, reinterpret_cast<hipStream_t>(stream)),
                 "ncclAllReduce");
  }

  int nranks() const { return nranks_; }
  int rank() const { return rank_; }
  uintptr_t handle() const { return reinterpret_cast<uintptr_t>(comm_); }

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_;
};

}  // namespace dcg_comm
