// Device parse of one JSON number token (json_parse.hip, json_span.hip): the host parser's
// grammar and arithmetic for the "simple" rows the workers' pre-scan admits (numbers made of
// [0-9.-] only, at most 16 characters: Clinger's fast path in fp64 -- both operands exact, one
// correctly rounded IEEE op -- or an exact u64 -> f64 for plain integers), so the result is
// bit-exact with Python's float() (the reference's json.loads, README.md:54,74).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tkh {
namespace {

__device__ __forceinline__ bool is_sep(uint32_t c) {
  return c == ',' || c == ' ' || c == '[' || c == ']' || c == '\n' || c == '\t' || c == '\r';
}

__device__ __constant__ double kP10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                           1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// The token starting at window byte s, parsed from registers: the 32 LDS bytes from
// s & ~15 (two ds_read_b128) are funnel-shifted so that t[0..4] hold bytes s .. s+19, and a
// fully unrolled walk over at most 17 bytes (a simple row's number has <= 16 characters,
// then a separator) runs the host parser's grammar with no dependent memory access.
// `avail` = bytes of the window from s on.  Returns 1 ok, 0 grammar error, 2 cut by the
// window end (parsed again in the next window).
__device__ __forceinline__ int parse_token_regs(const uint8_t* buf, int s, int avail, bool last_window, float* out) {
  const int A = s & ~15;
  // two whole ds_read_b128 (nontemporal: a no-op hint for LDS that keeps the compiler from
  // narrowing them to the dwords it can prove are used, as ds_read2_b32 pairs)
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u lv = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(buf + A));
  const v4u hv = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(buf + A + 16));
  const uint4 lo = make_uint4(lv.x, lv.y, lv.z, lv.w), hi = make_uint4(hv.x, hv.y, hv.z, hv.w);
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  const int o = s - A, q = o >> 2;
  const uint32_t sh = uint32_t(o & 3) * 8u;
  uint32_t t[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    // dwords q+k and q+k+1 (q <= 3, so at most w[7] and a dummy)
    const uint32_t a0 = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
    const uint32_t a1 = q == 0 ? w[k + 1] : q == 1 ? w[k + 2] : q == 2 ? w[k + 3] : (k + 4 < 8 ? w[k + 4] : 0u);
    t[k] = sh ? (a0 >> sh) | (a1 << (32u - sh)) : a0;
  }
  bool neg = false, dot = false, frac = false, any = false, ended = false, bad = false, truncated = false;
  uint32_t endc = 0;
  int endj = 17;
  uint64_t mant = 0;
  int nd = 0, exp10 = 0;
#pragma unroll
  for (int j = 0; j < 17; ++j) {
    const uint32_t c = (t[j >> 2] >> ((j & 3) * 8)) & 0xFFu;
    if (!ended) {
      if (j >= avail) {
        ended = true;
        endj = j;
        endc = 0x100u;  // window end
      } else if (j == 0 && c == '-') {
        neg = true;
      } else if (c - '0' <= 9u) {
        const uint32_t dd = c - '0';
        any = true;
        if (dot) frac = true;
        if (mant == 0 && dd == 0) {
          if (dot) --exp10;
        } else if (nd < 19) {
          mant = mant * 10 + dd;
          ++nd;
          if (dot) --exp10;
        } else {
          truncated = true;
          if (!dot) ++exp10;
        }
      } else if (c == '.' && !dot) {
        dot = true;
      } else {
        ended = true;
        endj = j;
        endc = c;
      }
    }
  }
  if (!ended) return 3;  // 17 number characters: longer than a simple number (json_scan_simple's run rule)
  if (endc == 0x100u) {
    if (!last_window) return 2;
    return 0;  // text ended inside a number
  }
  (void)endj;
  bad = !any || (dot && !frac) || !is_sep(endc);
  if (bad) return 0;
  if (mant == 0 && !dot) neg = false;  // "-0" is the JSON integer 0: +0.0 after Python's float()
  double v;
  if (!truncated && mant <= (uint64_t(1) << 53) && exp10 >= -22 && exp10 <= 22) {
    v = exp10 < 0 ? double(mant) / kP10[-exp10] : double(mant) * kP10[exp10];
  } else if (!truncated && exp10 == 0) {
    v = double(mant);  // one rounding: the hi/lo u32 halves convert exactly, the add rounds
  } else {
    return 0;  // the worker's pre-scan never sends such tokens
  }
  *out = float(neg ? -v : v);
  return 1;
}

}  // namespace
}  // namespace tkh
