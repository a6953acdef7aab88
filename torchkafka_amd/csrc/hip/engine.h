#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

namespace tkh {

class Engine {
 public:
  Engine(int device, int n_slots, size_t staging_bytes);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  int device() const { return device_; }
  int n_slots() const { return n_slots_; }
  size_t staging_stride() const { return stride_; }
  void* staging(int s) const { return static_cast<uint8_t*>(staging_) + stride_ * size_t(s); }
  hipStream_t copy_stream() const { return copy_stream_; }

  void register_host(void* p, size_t len);
  void unregister_host();
  bool host_registered() const { return host_ptr_ != nullptr; }

  void h2d(int s, const void* host, size_t nbytes);
  bool h2d_complete(int s);
  void wait_h2d(int s);
  void collate_fixed(int s, hipStream_t stream, size_t values_offset, int src_dt, void* dst, int dst_dt, int64_t rows,
                     int64_t row, const float* shift, const float* scale);
  void collate_varlen(int s, hipStream_t stream, size_t values_offset, int src_dt, void* out, int dst_dt, int64_t rows,
                      int64_t L, double pad, int64_t* lengths, uint8_t* mask);
  void copy_raw(int s, hipStream_t stream, size_t offset, void* dst, size_t nbytes);
  void synchronize();

 private:
  void check_slot(int s) const;
  int device_;
  int n_slots_;
  size_t stride_ = 0;
  void* staging_ = nullptr;
  hipStream_t copy_stream_ = nullptr;
  std::vector<hipEvent_t> h2d_done_, consumed_;
  void* host_ptr_ = nullptr;
  size_t host_len_ = 0;
};

}  // namespace tkh
