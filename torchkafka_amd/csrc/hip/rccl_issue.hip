// Device side of the native RCCL lockstep transport (rccl_lockstep.h): the agreement words' copy
// kernel and issue(), which launches it around RCCL's all-reduce.  The rest is host code
// (rccl_lockstep.cpp).
#include <hip/hip_runtime.h>

#include "rccl_lockstep.h"

#include <rccl/rccl.h>

#include <chrono>
#include <stdexcept>
#include <string>

#include "rccl_api.h"

namespace tkh {

namespace {

// The agreement's words between pinned host memory and the device buffer RCCL reduces: one wave,
// one word per lane (system-coherent host-mapped memory, read and written over PCIe).
__global__ void words_copy_kernel(const int64_t* __restrict__ src, int64_t* __restrict__ dst, int n) {
  const int i = int(threadIdx.x);
  if (i < n) dst[i] = src[i];
}

int64_t steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace

int RcclLockstep::issue(const int64_t in[kW]) {
  const int64_t t_issue = tracing_ ? steady_ns() : 0;
  const int s = int(issued_ % uint64_t(slots_));
  if (aborted_) throw std::runtime_error("lockstep: the RCCL communicator was aborted after a failure");
  // the slot's previous round trip must be complete before its buffers are reused
  wait_event(s, "lockstep slot reuse");
  int64_t* hin = h_in_ + kW * s;
  int64_t* hout = h_out_ + kW * s;
  int64_t* din = d_ + 2 * kW * s;
  int64_t* dout = din + kW;
  for (int k = 0; k < kW; ++k) hin[k] = in[k];
  auto* comm = static_cast<ncclComm_t>(comm_);
  if (mode_ == 1) {
    // RCCL reads and writes the host-mapped words itself: one queue operation
    check(api_, api_->AllReduce(h_in_dev_ + kW * s, h_out_dev_ + kW * s, kW, ncclInt64, ncclMin, comm, stream_),
          "ncclAllReduce");
  } else if (mode_ == 2) {
    TKH_HIP(hipMemcpyAsync(din, hin, kW * sizeof(int64_t), hipMemcpyHostToDevice, stream_));
    check(api_, api_->AllReduce(din, dout, kW, ncclInt64, ncclMin, comm, stream_), "ncclAllReduce");
    TKH_HIP(hipMemcpyAsync(hout, dout, kW * sizeof(int64_t), hipMemcpyDeviceToHost, stream_));
  } else if (mode_ == 3) {
    // the three dependent operations below, captured once per slot: one submission per agreement
    TKH_HIP(hipGraphLaunch(static_cast<hipGraphExec_t>(graphs_[size_t(s)]), stream_));
  } else {
    hipLaunchKernelGGL(words_copy_kernel, dim3(1), dim3(64), 0, stream_, h_in_dev_ + kW * s, din, kW);
    TKH_HIP(hipGetLastError());
    check(api_, api_->AllReduce(din, dout, kW, ncclInt64, ncclMin, comm, stream_), "ncclAllReduce");
    hipLaunchKernelGGL(words_copy_kernel, dim3(1), dim3(64), 0, stream_, dout, h_out_dev_ + kW * s, kW);
    TKH_HIP(hipGetLastError());
  }
  TKH_HIP(hipEventRecord(ev_[size_t(s)], stream_));
  ++issued_;
  if (tracing_ && trace_.size() < (size_t(1) << 20)) {
    slot_rec_[size_t(s)] = int64_t(trace_.size());
    trace_.push_back(TraceRec{t_issue, steady_ns(), 0, 0});
  }
  return s;
}

// TORCHKAFKA_RCCL_WORDS=graph: words in, RCCL's all-reduce and words out captured into one HIP
// graph per slot (their buffers are the slot's, fixed), so an agreement is one hipGraphLaunch
// instead of three launches.  Any capture failure falls back to the three launches.
void RcclLockstep::capture_graphs() {
  auto* comm = static_cast<ncclComm_t>(comm_);
  graphs_.assign(size_t(slots_), nullptr);
  for (int s = 0; s < slots_; ++s) {
    int64_t* din = d_ + 2 * kW * s;
    int64_t* dout = din + kW;
    hipGraph_t g = nullptr;
    bool ok = hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal) == hipSuccess;
    if (ok) {
      hipLaunchKernelGGL(words_copy_kernel, dim3(1), dim3(64), 0, stream_, h_in_dev_ + kW * s, din, kW);
      ok = hipGetLastError() == hipSuccess;
      ok = api_->AllReduce(din, dout, kW, ncclInt64, ncclMin, comm, stream_) == ncclSuccess && ok;
      hipLaunchKernelGGL(words_copy_kernel, dim3(1), dim3(64), 0, stream_, dout, h_out_dev_ + kW * s, kW);
      ok = hipGetLastError() == hipSuccess && ok;
      ok = hipStreamEndCapture(stream_, &g) == hipSuccess && ok && g != nullptr;
    }
    hipGraphExec_t ex = nullptr;
    if (ok) ok = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) == hipSuccess;
    if (g) (void)hipGraphDestroy(g);
    if (!ok) {
      (void)hipGetLastError();
      release_graphs();
      graph_fallback_ = true;
      mode_ = 0;
      return;
    }
    graphs_[size_t(s)] = ex;
  }
}

void RcclLockstep::release_graphs() {
  for (void* g : graphs_)
    if (g) (void)hipGraphExecDestroy(static_cast<hipGraphExec_t>(g));
  graphs_.clear();
}

}  // namespace tkh
