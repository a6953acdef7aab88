// Element types handled by the collate kernels and their conversions.
//
// Conversions are bit-exact with PyTorch's `Tensor.to(dtype)` on the same
// values (the numerics tests compare against it):
//   f32 -> bf16 : round-to-nearest-even; a plain `(__bf16)` cast lowers to
//                 v_cvt_pk_bf16_f32 on gfx950, which keeps NaNs NaN
//                 (MI355X_MICROARCH.md "Correctness boundaries").
//   f32 -> f16  : RNE via `(_Float16)`.
//   f32 -> fp8  : OCP e4m3fn (NOT the MI300 fnuz encoding), reproducing
//                 c10::detail::fp8e4m3fn_from_fp32_value: RNE, values whose
//                 magnitude rounds past 448 become NaN (0x7F | sign).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tkh {

enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2, kFP8E4M3 = 3, kU8 = 4, kI8 = 5, kI32 = 6, kI64 = 7, kBool = 8 };

inline int dtype_size(int dt) {
  switch (dt) {
    case kF32: case kI32: return 4;
    case kF16: case kBF16: return 2;
    case kFP8E4M3: case kU8: case kI8: case kBool: return 1;
    case kI64: return 8;
    default: return 0;
  }
}

struct fp8e4m3 { uint8_t bits; };

__host__ __device__ __forceinline__ uint8_t f32_to_fp8e4m3fn(float f) {
  constexpr uint32_t fp8_max = 1087u << 20;      // 480.0f: first value not representable
  constexpr uint32_t denorm_mask = 141u << 23;   // ((127 - 7) + (23 - 3) + 1)
  uint32_t bits = __builtin_bit_cast(uint32_t, f);
  const uint32_t sign = bits & 0x80000000u;
  bits ^= sign;
  uint8_t r;
  if (bits >= fp8_max) {
    r = 0x7F;
  } else if (bits < (121u << 23)) {
    // below the smallest normal (2^-6): add a magic constant so the FPU's
    // round-to-nearest-even places the denormal mantissa in the low bits
    const uint32_t t = __builtin_bit_cast(uint32_t, __builtin_bit_cast(float, bits) + __builtin_bit_cast(float, denorm_mask));
    r = uint8_t(t - denorm_mask);
  } else {
    const uint32_t mant_odd = (bits >> 20) & 1u;
    bits += ((uint32_t)(7 - 127) << 23) + 0x7FFFFu;
    bits += mant_odd;
    r = uint8_t(bits >> 20);
  }
  return r | uint8_t(sign >> 24);
}

// ---- load any source element as f32 (float path) or int64 (integer path)
template <typename S> __device__ __forceinline__ float to_f32(S v) { return float(v); }
template <> __device__ __forceinline__ float to_f32<__bf16>(__bf16 v) { return float(v); }
template <> __device__ __forceinline__ float to_f32<_Float16>(_Float16 v) { return float(v); }

template <typename D> struct Store;
template <> struct Store<float> { __host__ __device__ static float cvt(float v) { return v; } };
template <> struct Store<__bf16> { __host__ __device__ static __bf16 cvt(float v) { return (__bf16)v; } };
template <> struct Store<_Float16> { __host__ __device__ static _Float16 cvt(float v) { return (_Float16)v; } };
template <> struct Store<fp8e4m3> { __host__ __device__ static fp8e4m3 cvt(float v) { return fp8e4m3{f32_to_fp8e4m3fn(v)}; } };

}  // namespace tkh
