// H2D engine: pinned-ring registration, side-stream hipMemcpyAsync, per-slot
// events and the collate launches.
//
// Per ring slot s the engine owns a device staging buffer staging[s] and two
// events:
//   h2d_done[s]  recorded on the copy stream after the H2D copy of slot s;
//                the compute stream waits on it before the collate kernel and
//                the host polls it to recycle the host slot early (the pinned
//                slot is free as soon as the DMA read it, not after the kernel);
//   consumed[s]  recorded on the compute stream after the collate kernel;
//                the copy stream waits on it before overwriting staging[s].
// No allocation, no synchronisation in the per-batch path (Guideline 9).
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "collate.h"
#include "engine.h"

namespace tkh {

#define TKH_CHECK(expr)                                                                       \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

Engine::Engine(int device, int n_slots, size_t staging_bytes) : device_(device), n_slots_(n_slots) {
  if (n_slots <= 0) throw std::invalid_argument("engine: n_slots must be positive");
  TKH_CHECK(hipSetDevice(device_));
  TKH_CHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
  stride_ = (staging_bytes + 256 + 4095) / 4096 * 4096;
  TKH_CHECK(hipMalloc(&staging_, stride_ * size_t(n_slots)));
  h2d_done_.resize(size_t(n_slots));
  consumed_.resize(size_t(n_slots));
  for (int i = 0; i < n_slots; ++i) {
    TKH_CHECK(hipEventCreateWithFlags(&h2d_done_[size_t(i)], hipEventDisableTiming));
    TKH_CHECK(hipEventCreateWithFlags(&consumed_[size_t(i)], hipEventDisableTiming));
  }
}

Engine::~Engine() {
  hipSetDevice(device_);
  hipStreamSynchronize(copy_stream_);
  if (host_ptr_) hipHostUnregister(host_ptr_);
  for (auto e : h2d_done_) hipEventDestroy(e);
  for (auto e : consumed_) hipEventDestroy(e);
  if (staging_) hipFree(staging_);
  hipStreamDestroy(copy_stream_);
}

void Engine::check_slot(int s) const {
  if (s < 0 || s >= n_slots_) throw std::out_of_range("engine: bad slot");
}

void Engine::register_host(void* p, size_t len) {
  if (host_ptr_) throw std::runtime_error("engine: a host region is already registered");
  TKH_CHECK(hipSetDevice(device_));
  TKH_CHECK(hipHostRegister(p, len, hipHostRegisterDefault));
  host_ptr_ = p;
  host_len_ = len;
}

void Engine::unregister_host() {
  if (!host_ptr_) return;
  TKH_CHECK(hipStreamSynchronize(copy_stream_));
  TKH_CHECK(hipHostUnregister(host_ptr_));
  host_ptr_ = nullptr;
  host_len_ = 0;
}

void Engine::h2d(int s, const void* host, size_t nbytes) {
  check_slot(s);
  if (nbytes + 256 > stride_) throw std::invalid_argument("engine: copy larger than the staging buffer");
  // staging[s] may still be read by the previous batch's collate kernel
  TKH_CHECK(hipStreamWaitEvent(copy_stream_, consumed_[size_t(s)], 0));
  if (nbytes) TKH_CHECK(hipMemcpyAsync(staging(s), host, nbytes, hipMemcpyHostToDevice, copy_stream_));
  TKH_CHECK(hipEventRecord(h2d_done_[size_t(s)], copy_stream_));
}

bool Engine::h2d_complete(int s) {
  check_slot(s);
  hipError_t e = hipEventQuery(h2d_done_[size_t(s)]);
  if (e == hipSuccess) return true;
  if (e == hipErrorNotReady) return false;
  throw std::runtime_error(std::string("engine: h2d event: ") + hipGetErrorString(e));
}

void Engine::wait_h2d(int s) {
  check_slot(s);
  TKH_CHECK(hipEventSynchronize(h2d_done_[size_t(s)]));
}

void Engine::collate_fixed(int s, hipStream_t stream, size_t values_offset, int src_dt, void* dst, int dst_dt,
                           int64_t rows, int64_t row, const float* shift, const float* scale) {
  check_slot(s);
  TKH_CHECK(hipStreamWaitEvent(stream, h2d_done_[size_t(s)], 0));
  launch_fixed(static_cast<uint8_t*>(staging(s)) + values_offset, src_dt, dst, dst_dt, rows, row, shift, scale, stream);
  TKH_CHECK(hipEventRecord(consumed_[size_t(s)], stream));
}

void Engine::collate_varlen(int s, hipStream_t stream, size_t values_offset, int src_dt, void* out, int dst_dt,
                            int64_t rows, int64_t L, double pad, int64_t* lengths, uint8_t* mask) {
  check_slot(s);
  TKH_CHECK(hipStreamWaitEvent(stream, h2d_done_[size_t(s)], 0));
  auto* base = static_cast<uint8_t*>(staging(s));
  launch_varlen(reinterpret_cast<const int32_t*>(base), base + values_offset, src_dt, out, dst_dt, rows, L, pad,
                lengths, mask, stream);
  TKH_CHECK(hipEventRecord(consumed_[size_t(s)], stream));
}

void Engine::copy_raw(int s, hipStream_t stream, size_t offset, void* dst, size_t nbytes) {
  check_slot(s);
  TKH_CHECK(hipStreamWaitEvent(stream, h2d_done_[size_t(s)], 0));
  if (nbytes)
    TKH_CHECK(hipMemcpyAsync(dst, static_cast<uint8_t*>(staging(s)) + offset, nbytes, hipMemcpyDeviceToDevice, stream));
  TKH_CHECK(hipEventRecord(consumed_[size_t(s)], stream));
}

void Engine::synchronize() { TKH_CHECK(hipStreamSynchronize(copy_stream_)); }

}  // namespace tkh
