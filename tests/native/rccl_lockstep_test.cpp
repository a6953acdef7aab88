// Host test of the RCCL lockstep transport's failure detection (csrc/hip/rccl_lockstep.cpp,
// VERDICT r5 do-this 6): the bounded wait that aborts the communicator when a peer never answers,
// the asynchronous-error branch, a failing event, and the teardown after an abort.  No GPU and no
// second rank: the HIP runtime calls are stubbed below (an agreement "completes" when the test says
// so) and RCCL is a stub library (rccl_stub.cpp) the transport dlopen()s like the real one.
// Run by tools/sanitize.sh under AddressSanitizer + UBSan.  Usage: rccl_lockstep_test <stub.so>
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "rccl_lockstep.h"
#include "reaper.h"

// ---- stubbed HIP runtime (what the host half calls)
static hipError_t g_query = hipErrorNotReady;  // what every hipEventQuery returns
static int g_events = 0, g_syncs = 0, g_host_frees = 0, g_dev_frees = 0;
extern "C" {
hipError_t hipSetDevice(int) { return hipSuccess; }
const char* hipGetErrorString(hipError_t e) { return e == hipErrorLaunchFailure ? "launch failure (stub)" : "stub"; }
hipError_t hipDeviceGetStreamPriorityRange(int* l, int* g) {
  *l = 0;
  *g = -1;
  return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) {
  *s = reinterpret_cast<hipStream_t>(0x2000);
  return hipSuccess;
}
hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned, int) {
  *s = reinterpret_cast<hipStream_t>(0x2001);
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) {
  ++g_syncs;
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
hipError_t hipMalloc(void** p, size_t n) {
  *p = std::calloc(1, n);
  return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t n, unsigned) {
  *p = std::calloc(1, n);
  return hipSuccess;
}
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) {
  *d = h;
  return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  *e = reinterpret_cast<hipEvent_t>(static_cast<intptr_t>(0x3000 + ++g_events));
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return g_query; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
  std::memmove(d, s, n);
  return hipSuccess;
}
}
namespace tkh {
// the device half (rccl_issue.hip: the words kernel around the all-reduce) is not built here
int RcclLockstep::issue(const int64_t*) { throw std::logic_error("issue() is device code"); }
void RcclLockstep::capture_graphs() {}
void RcclLockstep::release_graphs() { graphs_.clear(); }
// the deferred-release thread: released at once here
void Reaper::free_device(int, void* p) {
  ++g_dev_frees;
  std::free(p);
}
void Reaper::free_host(int, void* p) {
  ++g_host_frees;
  std::free(p);
}
}  // namespace tkh

#define CHECK(c)                                                                          \
  do {                                                                                    \
    if (!(c)) {                                                                           \
      std::fprintf(stderr, "rccl_lockstep_test FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

template <class F>
static std::string raises(F f) {
  try {
    f();
  } catch (const std::exception& e) {
    return e.what();
  }
  return "";
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string lib = argv[1];
  void* h = dlopen(lib.c_str(), RTLD_NOW | RTLD_GLOBAL);
  CHECK(h != nullptr);
  int* async_error = static_cast<int*>(dlsym(h, "stub_async_error"));
  int* aborts = static_cast<int*>(dlsym(h, "stub_aborts"));
  int* destroys = static_cast<int*>(dlsym(h, "stub_destroys"));
  CHECK(async_error && aborts && destroys);
  const std::string id = tkh::RcclLockstep::unique_id(lib);
  CHECK(id.size() == 128);
  int64_t out[tk::kLockstepWords];
  using clk = std::chrono::steady_clock;

  // 1. a peer that never answers: the wait gives up after the timeout, aborts the communicator
  //    and raises; every later call raises at once; the teardown neither waits nor destroys it
  {
    auto* ls = new tkh::RcclLockstep(lib, id, 0, 2, 0, 4);
    CHECK(ls->comm_count() == 2);
    ls->set_timeout_ms(60);
    g_query = hipErrorNotReady;
    const auto t0 = clk::now();
    const std::string e = raises([&] { ls->wait(0, out); });
    const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    CHECK(e.find("no answer from the other ranks within 60 ms") != std::string::npos);
    CHECK(ms >= 55 && ms < 2000);
    CHECK(*aborts == 1 && ls->aborted());
    CHECK(raises([&] { ls->wait(1, out); }).find("aborted") != std::string::npos);
    CHECK(raises([&] { ls->allreduce_sum(1); }).find("aborted") != std::string::npos);
    CHECK(raises([&] { (void)ls->comm_count(); }).find("aborted") != std::string::npos);
    const int syncs = g_syncs, destroyed = *destroys;
    delete ls;  // no stream synchronize (the collective may never end), no destroy of an aborted comm
    CHECK(g_syncs == syncs && *destroys == destroyed);
    CHECK(g_dev_frees == 1 && g_host_frees == 2);
  }
  // 2. RCCL reports an asynchronous error (a peer failed): raised well before the timeout
  {
    tkh::RcclLockstep ls(lib, id, 0, 2, 0, 4);
    ls.set_timeout_ms(60000);
    *async_error = int(ncclRemoteError);
    g_query = hipErrorNotReady;
    const auto t0 = clk::now();
    const std::string e = raises([&] { ls.wait(2, out); });
    const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    CHECK(e.find("asynchronous error") != std::string::npos && e.find("stub remote error") != std::string::npos);
    CHECK(ms < 1000);
    CHECK(*aborts == 2 && ls.aborted());
    *async_error = int(ncclSuccess);
  }
  // 3. ncclInProgress is not a failure: the wait goes on to its timeout
  {
    tkh::RcclLockstep ls(lib, id, 0, 2, 0, 4);
    ls.set_timeout_ms(40);
    *async_error = int(ncclInProgress);
    g_query = hipErrorNotReady;
    CHECK(raises([&] { ls.wait(0, out); }).find("within 40 ms") != std::string::npos);
    *async_error = int(ncclSuccess);
  }
  // 4. a failing event is raised as such (no abort: the runtime failed, not a peer)
  {
    tkh::RcclLockstep ls(lib, id, 0, 2, 0, 4);
    g_query = hipErrorLaunchFailure;
    const int a0 = *aborts;
    CHECK(raises([&] { ls.wait(1, out); }).find("launch failure (stub)") != std::string::npos);
    CHECK(*aborts == a0 && !ls.aborted());
  }
  // 5. agreements that complete: results come back, start-up sum, normal teardown destroys the comm
  {
    const int d0 = *destroys;
    {
      tkh::RcclLockstep ls(lib, id, 0, 2, 0, 4);
      g_query = hipSuccess;
      CHECK(ls.ready(0));
      ls.wait(0, out);
      CHECK(ls.allreduce_sum(41) == 41);  // the stub's "all-reduce" of one rank's word
    }
    CHECK(*destroys == d0 + 1);
  }
  std::printf("rccl_lockstep_test: ok\n");
  return 0;
}
