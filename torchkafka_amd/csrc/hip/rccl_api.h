// Internal to the RCCL lockstep transport (rccl_lockstep.cpp host side, rccl_issue.hip device
// side): the RCCL entry points resolved with dlopen() and the error helpers both halves use.
#pragma once
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <stdexcept>
#include <string>

#include "lockstep.h"

namespace tkh {

struct RcclApi {
  void* lib = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;                         // optional
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;  // optional
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

#define TKH_HIP(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

inline void check(RcclApi* api, ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + api->GetErrorString(r));
}

constexpr int kW = tk::kLockstepWords;

}  // namespace tkh
