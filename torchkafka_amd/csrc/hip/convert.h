// Element conversions shared by the gfx950 kernels (collate.hip, span_decode.hip): source
// element -> destination element, bit-exact with torch's Tensor.to (dtypes.h), with the
// optional fused (x - shift) * scale normalisation on float destinations.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dtypes.h"

namespace tkh {

template <typename T, int N>
struct alignas(sizeof(T) * N >= 16 ? 16 : sizeof(T) * N) Vec {
  T v[N];
};

// ---------------------------------------------------------------- conversion
template <typename S, typename D, bool IntPath>
struct Conv;

template <typename S, typename D>
struct Conv<S, D, false> {  // float destination
  __device__ __forceinline__ static D apply(S s, float shift, float scale, bool affine) {
    float x = to_f32<S>(s);
    if (affine) x = (x - shift) * scale;
    return Store<D>::cvt(x);
  }
};
template <typename S, typename D>
struct Conv<S, D, true> {  // integer destination (token ids etc.)
  __device__ __forceinline__ static D apply(S s, float, float, bool) { return D(int64_t(s)); }
};

template <typename D> struct IsIntDst { static constexpr bool value = false; };
template <> struct IsIntDst<int32_t> { static constexpr bool value = true; };
template <> struct IsIntDst<int64_t> { static constexpr bool value = true; };
template <> struct IsIntDst<uint8_t> { static constexpr bool value = true; };

inline bool is_float_dt(int dt) { return dt == kF32 || dt == kF16 || dt == kBF16 || dt == kFP8E4M3; }

}  // namespace tkh

// Runtime dtype codes -> template instantiation: FN<S, D>(...) for (src_dt, dst_dt) in scope.
#define TK_DISPATCH_DST(S, FN, ...)                                                    \
  switch (dst_dt) {                                                                    \
    case kF32: FN<S, float>(__VA_ARGS__); break;                                       \
    case kF16: FN<S, _Float16>(__VA_ARGS__); break;                                    \
    case kBF16: FN<S, __bf16>(__VA_ARGS__); break;                                     \
    case kFP8E4M3: FN<S, fp8e4m3>(__VA_ARGS__); break;                                 \
    case kI32: FN<S, int32_t>(__VA_ARGS__); break;                                     \
    case kI64: FN<S, int64_t>(__VA_ARGS__); break;                                     \
    default: throw std::invalid_argument("collate: unsupported destination dtype");    \
  }

#define TK_DISPATCH_SRC(FN, ...)                                                       \
  switch (src_dt) {                                                                    \
    case kF32: TK_DISPATCH_DST(float, FN, __VA_ARGS__) break;                          \
    case kF16: TK_DISPATCH_DST(_Float16, FN, __VA_ARGS__) break;                       \
    case kBF16: TK_DISPATCH_DST(__bf16, FN, __VA_ARGS__) break;                        \
    case kU8: TK_DISPATCH_DST(uint8_t, FN, __VA_ARGS__) break;                         \
    case kI8: TK_DISPATCH_DST(int8_t, FN, __VA_ARGS__) break;                          \
    case kI32: TK_DISPATCH_DST(int32_t, FN, __VA_ARGS__) break;                        \
    case kI64: TK_DISPATCH_DST(int64_t, FN, __VA_ARGS__) break;                        \
    default: throw std::invalid_argument("collate: unsupported source dtype");         \
  }
