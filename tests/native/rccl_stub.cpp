// A stand-in librccl for tests/native/rccl_lockstep_test.cpp: the entry points the RCCL lockstep
// transport resolves with dlopen() (csrc/hip/rccl_api.h), driven by the stub_* globals the test sets.
#include <rccl/rccl.h>

#include <cstring>

extern "C" {
int stub_async_error = 0;  // what ncclCommGetAsyncError reports
int stub_aborts = 0, stub_destroys = 0, stub_allreduces = 0, stub_inits = 0;

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::memset(id->internal, 7, sizeof(id->internal));
  return ncclSuccess;
}
ncclResult_t ncclCommInitRank(ncclComm_t* c, int, ncclUniqueId, int) {
  ++stub_inits;
  *c = reinterpret_cast<ncclComm_t>(0x1000);
  return ncclSuccess;
}
ncclResult_t ncclAllReduce(const void* s, void* d, size_t n, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) {
  ++stub_allreduces;
  std::memmove(d, s, n * 8);  // world "1": the result is the input (host memory in the test)
  return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t) {
  ++stub_destroys;
  return ncclSuccess;
}
ncclResult_t ncclCommCount(const ncclComm_t, int* n) {
  *n = 2;
  return ncclSuccess;
}
ncclResult_t ncclCommAbort(ncclComm_t) {
  ++stub_aborts;
  return ncclSuccess;
}
ncclResult_t ncclCommGetAsyncError(ncclComm_t, ncclResult_t* e) {
  *e = static_cast<ncclResult_t>(stub_async_error);
  return ncclSuccess;
}
const char* ncclGetErrorString(ncclResult_t) { return "stub remote error"; }
}
