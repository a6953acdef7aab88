// Host side of the native RCCL lockstep transport (rccl_lockstep.h): the communicator, the bounded
// waits with failure detection, the start-up checks.  Plain HIP runtime calls only -- the one
// device kernel (the agreement words' copy) and issue() are in rccl_issue.hip -- so this file
// also builds for the host test with the HIP and RCCL symbols stubbed (tests/native/rccl_lockstep_test.cpp).
#include "rccl_lockstep.h"

#include "rccl_api.h"
#include "reaper.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace tkh {

namespace {

RcclApi* load_api(const std::string& path) {
  // Prefer the instance already in the process (torch's), then the given path, then the system one.
  void* lib = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
  if (!lib) lib = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!lib) lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) throw std::runtime_error(std::string("cannot load RCCL: ") + dlerror());
  auto* api = new RcclApi();
  api->lib = lib;
  auto sym = [&](const char* name) {
    void* p = dlsym(lib, name);
    if (!p) throw std::runtime_error(std::string("RCCL symbol missing: ") + name);
    return p;
  };
  api->GetUniqueId = reinterpret_cast<decltype(api->GetUniqueId)>(sym("ncclGetUniqueId"));
  api->CommInitRank = reinterpret_cast<decltype(api->CommInitRank)>(sym("ncclCommInitRank"));
  api->AllReduce = reinterpret_cast<decltype(api->AllReduce)>(sym("ncclAllReduce"));
  api->CommDestroy = reinterpret_cast<decltype(api->CommDestroy)>(sym("ncclCommDestroy"));
  api->CommCount = reinterpret_cast<decltype(api->CommCount)>(sym("ncclCommCount"));
  api->GetErrorString = reinterpret_cast<decltype(api->GetErrorString)>(sym("ncclGetErrorString"));
  api->CommAbort = reinterpret_cast<decltype(api->CommAbort)>(dlsym(lib, "ncclCommAbort"));
  api->CommGetAsyncError = reinterpret_cast<decltype(api->CommGetAsyncError)>(dlsym(lib, "ncclCommGetAsyncError"));
  return api;
}

int words_mode_env() {
  const char* e = std::getenv("TORCHKAFKA_RCCL_WORDS");
  if (!e) return 0;
  const std::string v(e);
  return v == "host" ? 1 : v == "copy" ? 2 : v == "graph" ? 3 : 0;
}

}  // namespace

std::string RcclLockstep::unique_id(const std::string& lib_path) {
  RcclApi* api = load_api(lib_path);
  ncclUniqueId id;
  check(api, api->GetUniqueId(&id), "ncclGetUniqueId");
  delete api;  // the library stays loaded (no dlclose)
  return std::string(id.internal, sizeof(id.internal));
}

RcclLockstep::RcclLockstep(const std::string& lib_path, const std::string& id, int rank, int world, int device,
                           int slots)
    : rank_(rank), world_(world), device_(device), slots_(slots < 2 ? 2 : slots) {
  if (id.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("RCCL unique id must be 128 bytes");
  const char* tr = std::getenv("TORCHKAFKA_LOCKSTEP_TRACE");
  tracing_ = tr && tr[0] == '1';
  slot_rec_.assign(size_t(slots_), -1);
  api_ = load_api(lib_path);
  TKH_HIP(hipSetDevice(device_));
  // At the device's greatest priority the lockstep's stream would get a hardware-queue pool of its
  // own (tools/probes/queue_probe.py), never sharing a queue with the decode streams.
  // Normal priority by default: on a queue of its own at the greatest priority an agreement took
  // ~110 µs to come back in the loop against ~60 µs on a normal one (profiles/r05_s19_rccl_matrix,
  // r05_s24); TORCHKAFKA_LOCKSTEP_PRIORITY=high restores the separate queue
  const char* pe = std::getenv("TORCHKAFKA_LOCKSTEP_PRIORITY");
  high_prio_ = pe && std::string(pe) == "high";
  if (high_prio_) {
    int least = 0, greatest = 0;
    TKH_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    TKH_HIP(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest));
  } else {
    TKH_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  }
  mode_ = words_mode_env();
  if (const char* pe = std::getenv("TORCHKAFKA_RCCL_POLL_EVERY")) poll_every_ = std::atoi(pe);
  TKH_HIP(hipMalloc(reinterpret_cast<void**>(&d_), sizeof(int64_t) * 2 * kW * size_t(slots_)));
  TKH_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_in_), sizeof(int64_t) * kW * size_t(slots_), hipHostMallocMapped));
  TKH_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_out_), sizeof(int64_t) * kW * size_t(slots_), hipHostMallocMapped));
  TKH_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_in_dev_), h_in_, 0));
  TKH_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_out_dev_), h_out_, 0));
  ev_.resize(size_t(slots_));
  for (auto& e : ev_) TKH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  ncclUniqueId uid;
  std::memcpy(uid.internal, id.data(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  check(api_, api_->CommInitRank(&comm, world_, uid, rank_), "ncclCommInitRank");
  comm_ = comm;
  if (mode_ == 3) capture_graphs();
}

RcclLockstep::~RcclLockstep() {
  (void)hipSetDevice(device_);
  if (!aborted_ && stream_) (void)hipStreamSynchronize(stream_);
  release_graphs();
  if (comm_) api_->CommDestroy(static_cast<ncclComm_t>(comm_));  // null once aborted
  for (auto e : ev_) (void)hipEventDestroy(e);
  Reaper::free_device(device_, d_);  // hipFree / hipHostFree wait for the whole device (reaper.h)
  Reaper::free_host(device_, h_in_);
  Reaper::free_host(device_, h_out_);
  if (stream_) (void)hipStreamDestroy(stream_);
  delete api_;
}

void RcclLockstep::wait_event(int t, const char* what) {
  hipEvent_t ev = ev_.at(size_t(t));
  hipError_t e = hipEventQuery(ev);
  if (e == hipSuccess) return;
  if (aborted_) throw std::runtime_error("lockstep: the RCCL communicator was aborted after a failure");
  // spin briefly (the round trip is normally done), then poll with short sleeps, checking
  // RCCL's asynchronous error state and the deadline
  const auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  for (;;) {
    e = hipEventQuery(ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
    if (++spins < 2000) continue;
    const auto el = std::chrono::steady_clock::now() - t0;
    const int64_t ms = std::chrono::duration_cast<std::chrono::milliseconds>(el).count();
    ncclResult_t async = ncclSuccess;
    if (api_->CommGetAsyncError) api_->CommGetAsyncError(static_cast<ncclComm_t>(comm_), &async);
    const bool failed = async != ncclSuccess && async != ncclInProgress;
    if (failed || (timeout_ms_ > 0 && ms > timeout_ms_)) {
      aborted_ = true;
      if (api_->CommAbort) api_->CommAbort(static_cast<ncclComm_t>(comm_));
      comm_ = nullptr;
      throw std::runtime_error(
          failed ? std::string("lockstep: RCCL reported an asynchronous error (") + api_->GetErrorString(async) +
                       "): a peer rank failed"
                 : "lockstep: no answer from the other ranks within " + std::to_string(timeout_ms_) +
                       " ms (a peer rank died or hung); RCCL communicator aborted");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

namespace {
int64_t steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

int RcclLockstep::comm_count() const {
  if (!comm_) throw std::runtime_error("lockstep: the RCCL communicator was aborted after a failure");
  int n = 0;
  check(api_, api_->CommCount(static_cast<ncclComm_t>(comm_), &n), "ncclCommCount");
  return n;
}

int64_t RcclLockstep::allreduce_sum(int64_t v) {
  if (aborted_) throw std::runtime_error("lockstep: the RCCL communicator was aborted after a failure");
  // every pipelined agreement is settled first: the slots' buffers are shared with issue()
  for (int s = 0; s < slots_; ++s) wait_event(s, "lockstep drain");
  const int s = int(issued_ % uint64_t(slots_));
  int64_t* hin = h_in_ + kW * s;
  int64_t* hout = h_out_ + kW * s;
  int64_t* din = d_ + 2 * kW * s;
  hin[0] = v;
  TKH_HIP(hipMemcpyAsync(din, hin, sizeof(int64_t), hipMemcpyHostToDevice, stream_));
  check(api_, api_->AllReduce(din, din + kW, 1, ncclInt64, ncclSum, static_cast<ncclComm_t>(comm_), stream_),
        "ncclAllReduce");
  TKH_HIP(hipMemcpyAsync(hout, din + kW, sizeof(int64_t), hipMemcpyDeviceToHost, stream_));
  TKH_HIP(hipEventRecord(ev_[size_t(s)], stream_));
  ++issued_;
  wait_event(s, "lockstep allreduce_sum");
  return hout[0];
}

bool RcclLockstep::ready(int t) { return hipEventQuery(ev_.at(size_t(t))) == hipSuccess; }

void RcclLockstep::wait(int t, int64_t out[kW]) {
  const int64_t w0 = tracing_ ? steady_ns() : 0;
  wait_event(t, "lockstep wait");
  if (tracing_ && slot_rec_.at(size_t(t)) >= 0 && size_t(slot_rec_[size_t(t)]) < trace_.size()) {
    TraceRec& r = trace_[size_t(slot_rec_[size_t(t)])];
    r.wait0 = w0;
    r.wait1 = steady_ns();
    slot_rec_[size_t(t)] = -1;
  }
  const volatile int64_t* hout = h_out_ + kW * t;
  for (int k = 0; k < kW; ++k) out[k] = hout[k];
}

}  // namespace tkh
