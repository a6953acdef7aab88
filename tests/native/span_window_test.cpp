// Host test of tk::SpanWindows (csrc/core/span.h), the window geometry the span kernels stream a
// log segment through (csrc/hip/span_device.h).  For every segment alignment (16 heads) and many
// lengths up to kSpanSegMax it checks that
//   * the windows' owned bytes partition the segment, and win_of() names the owner of each byte;
//   * a window stages 16-byte aligned chunks of the segment only, at most what its buffer holds;
//   * every read the kernels make for what a window owns lands inside its LDS buffer and, where the
//     bytes matter, on staged bytes: a 16-byte group starting in the window (span::lds16 reads the
//     two aligned slots around it), and every CRC lane's piece (a sliding dword window).
// Built and run under ASan/UBSan by tools/sanitize.sh (tests/test_sanitizers.py).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <initializer_list>

#include "span.h"

#define CHECK(c)                                                                          \
  do {                                                                                    \
    if (!(c)) {                                                                           \
      std::fprintf(stderr, "span_window_test FAILED %s:%d: %s -- ", __FILE__, __LINE__, #c); \
      std::fprintf(stderr, "head %d len %u k %d\n", head, len, k);                        \
      std::exit(1);                                                                       \
    }                                                                                     \
  } while (0)

static uint64_t check(int head, uint32_t len) {
  using namespace tk;
  int k = -1;
  const int32_t lo = 16 + head, hi = lo + int32_t(len);
  const SpanWindows W(lo, hi);
  CHECK(W.nw >= 1 && W.nw <= int32_t(kSpanMaxWins));
  CHECK(W.w0 <= lo && W.w0 + int32_t(kSpanWin) > lo);  // window 0 holds the first byte
  uint64_t reads = 0;
  for (k = 0; k < W.nw; ++k) {
    const int32_t a = W.own_lo(k), b = W.own_hi(k);
    CHECK(a < b);
    CHECK(k == 0 ? a == lo : a == W.own_hi(k - 1));
    if (k == W.nw - 1) CHECK(b == hi);
    CHECK(W.win_of(a) == k && W.win_of(b - 1) == k);
    const int32_t sl = W.stage_lo(k), sh = W.stage_hi(k);
    CHECK(sl % 16 == 0 && sh % 16 == 0 && sl >= 16 && sh <= ((hi + 15) & ~15) && sl < sh);
    CHECK(sh - sl <= int32_t(kSpanWin) + 96);
    // LDS byte of image byte x: kSpanWinPad + x - sl, inside [0, kSpanWinBytes)
    auto in_buf = [&](int32_t x) { return kSpanWinPad + x - sl >= 0 && kSpanWinPad + x - sl < kSpanWinBytes; };
    auto staged = [&](int32_t x) { return x >= sl && x < sh; };
    // 16-byte groups starting in the window (values, text pieces): bytes staged where they lie in
    // the segment, both aligned 16-byte slots of span::lds16 in the buffer
    for (int32_t b0 = a - 15; b0 < b; ++b0) {
      const int32_t key = b0 > lo ? b0 : lo;
      if (key < a || key >= b || b0 + 16 <= lo) continue;
      for (int32_t x = b0; x < b0 + 16; ++x)
        if (x >= lo && x < hi) CHECK(staged(x));
      if (b0 >= lo) {
        const int32_t l0 = kSpanWinPad + b0 - sl;
        CHECK((l0 & ~15) >= 0 && (l0 & ~15) + 32 <= kSpanWinBytes);
      }
      ++reads;
    }
    // CRC pieces of window k: lane t reads dwords from its piece start (when the piece reaches past
    // c0 - 4) to 8 bytes past its end; the bytes in [c0, hi) must be staged
    for (const int32_t c0 : {lo, lo + 21}) {
      if (c0 >= hi) continue;
      for (int32_t t = 0; t < int32_t(kSpanLanes); ++t) {
        const int32_t s = W.w0 + k * int32_t(kSpanWin) + t * int32_t(kSpanPiece), e = s + int32_t(kSpanPiece);
        CHECK(s >= a || k == 0);
        CHECK(e <= b || (k == 0 && e <= a + int32_t(kSpanWin)));
        if (e <= c0) continue;
        const int32_t first_read = (s + 4 > c0 ? s : s + 4 + 8 * ((c0 - s - 4) >> 3)) & ~3;
        CHECK(in_buf(first_read) && in_buf(e + 7));
        for (int32_t x = s > c0 ? s : c0; x < e; ++x) CHECK(staged(x));
      }
    }
  }
  return reads;
}

int main() {
  using namespace tk;
  uint64_t cases = 0, reads = 0;
  for (int head = 0; head < 16; ++head) {
    for (uint32_t len = 1; len < 200; ++len, ++cases) reads += check(head, len);
    for (uint32_t n = 1; n <= kSpanMaxWins; ++n)
      for (int d = -40; d <= 40; d += 3) {
        const int64_t len = int64_t(n) * kSpanWin + d;
        if (len >= 1 && len <= int64_t(kSpanSegMax)) {
          reads += check(head, uint32_t(len));
          ++cases;
        }
      }
    for (uint32_t len : {kSpanSegMax, kSpanSegMax - 1, 66'000u, 66'560u, 4096u}) {
      reads += check(head, len);
      ++cases;
    }
  }
  std::printf("span_window_test: ok (%llu segment shapes, %llu groups)\n", static_cast<unsigned long long>(cases),
              static_cast<unsigned long long>(reads));
  return 0;
}
