// One wave runs json_scan_simple's rules on a device-counted JSON row (csrc/core/consumer.cpp
// json_scan_impl, bit for bit).  Shared by json_span.hip's json_count_kernel (a wave per row, the
// width of a batch without pad_to needs every count before the parse) and json_parse.hip's
// json_rows_kernel (fixed pad_to width: the parse block counts its own row first).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace tkh {

__device__ __forceinline__ bool json_is_ws(uint32_t c) { return c == 32u || c == 9u || c == 10u || c == 13u; }

// The rules: whitespace trimmed, '[' ... ']' framing, an interior of number characters [0-9.-],
// commas and whitespace only, no run of more than 16 number characters.  load(c) gives the text's
// 16 bytes at c (c a multiple of 16; bytes past T are ignored), byte(i) its byte i.  Returns the
// element count (commas + 1; 0 for an empty interior), or -1 when the row is not simple; *guess is
// then the element count a flat array of that text has (commas + 1, 0 when the interior is empty or
// the text is not framed) -- the width its host parse will fill.  Every lane gets the result.
template <class Load, class Byte>
__device__ int32_t json_scan_row(Load&& load, Byte&& byte, int32_t T, int lane, int32_t* guess) {
  int32_t lo, hi;
  bool framed;
  if (T >= 2 && byte(0) == '[' && byte(T - 1) == ']') {
    lo = 1;
    hi = T - 1;
    framed = true;
  } else {
    int32_t fa = T, lb = -1;  // first and last byte that is not whitespace
    for (int32_t i = lane; i < T; i += 64)
      if (!json_is_ws(byte(i))) {
        fa = min(fa, i);
        lb = max(lb, i);
      }
#pragma unroll
    for (int off = 32; off; off >>= 1) {
      fa = min(fa, __shfl_xor(fa, off, 64));
      lb = max(lb, __shfl_xor(lb, off, 64));
    }
    framed = lb - fa + 1 >= 2 && byte(fa) == '[' && byte(lb) == ']';
    lo = framed ? fa + 1 : 0;
    hi = framed ? lb : 0;
  }
  int32_t commas = 0;
  bool bad = !framed, anyt = false, anyc = false;
  uint32_t carry = 0;  // number characters ending the previous 1 KiB pass (its lane 63)
  for (int32_t base = 0; base < T; base += 64 * 16) {
    const int32_t c = base + 16 * lane;
    uint32_t tokm = 0;
    if (c < T) {
      const uint4 v = load(c);
      const int32_t l0 = lo - c, h0 = hi - c;
      uint32_t in = h0 <= 0 ? 0u : h0 >= 16 ? 0xFFFFu : (1u << h0) - 1u;
      if (l0 > 0) in &= l0 >= 16 ? 0u : ~((1u << l0) - 1u);
      if (in) {
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
        uint32_t com = 0, oth = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const uint32_t ch = (wd[j >> 2] >> (8 * (j & 3))) & 0xFFu;
          const bool tk = ch - 48u <= 9u || ch == 46u || ch == 45u;
          tokm |= uint32_t(tk) << j;
          com |= uint32_t(ch == 44u) << j;
          oth |= uint32_t(!tk && ch != 44u && !json_is_ws(ch)) << j;
        }
        tokm &= in;
        com &= in;
        oth &= in;
        commas += __popc(com);
        bad = bad || oth != 0;
        anyt = anyt || tokm != 0;
        anyc = anyc || (tokm | com | oth) != 0;
      }
    }
    // a run of > 16 number characters crosses a chunk boundary (inside 16 bytes it cannot)
    const uint32_t lead = uint32_t(__builtin_ctz(~tokm));
    const uint32_t trail = uint32_t(__builtin_clz(~(tokm << 16)));
    uint32_t prev = __shfl_up(trail, 1, 64);
    if (lane == 0) prev = carry;
    if (prev + lead > 16u) bad = true;
    carry = __shfl(trail, 63, 64);
  }
#pragma unroll
  for (int off = 32; off; off >>= 1) commas += __shfl_xor(commas, off, 64);
  bad = __ballot(bad) != 0;
  anyt = __ballot(anyt) != 0;
  anyc = __ballot(anyc) != 0;
  *guess = framed && anyc ? commas + 1 : 0;
  if (bad) return -1;
  if (!anyt) return commas == 0 ? 0 : -1;
  return commas + 1;
}

}  // namespace tkh
