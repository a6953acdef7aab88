// Host test of tk::span_part (csrc/core/span.h), the byte ranges of a log segment decoded by 2 or 4
// workgroups (span_decode.hip step 0), run under AddressSanitizer + UBSan by tools/sanitize.sh.
// For every segment length (every length up to 4 KiB, then a stride up to kSpanSegMax) and both
// CRC starts: the parts' own ranges tile the segment in order; each part stages its own range, the
// 16 bytes of a value group starting at its end (or up to the segment's end) and stays inside the
// segment; and each CRC lane of the whole layout is run by exactly the part owning its bytes, which
// it staged.
#include <cstdio>
#include <cstdlib>
#include <initializer_list>

#include "span.h"

#define CHECK(c, ...)                                                   \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "span_split_test FAILED %s:%d: %s -- ", __FILE__, __LINE__, #c); \
      std::fprintf(stderr, __VA_ARGS__);                                \
      std::fprintf(stderr, "\n");                                       \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

static void check(uint32_t len, bool first, int P) {
  const int32_t n = int32_t(len), c0 = first ? 21 : 0;
  const int32_t L = int32_t(tk::span_lane_bytes(uint32_t(n - c0)));
  const int nl = int(tk::kSpanLanes) / P;
  int32_t prev = 0;
  for (int j = 0; j < P; ++j) {
    const tk::SpanPart p = tk::span_part(len, first, P, j);
    CHECK(p.own_lo == prev && p.own_lo <= p.own_hi, "len %u first %d P %d part %d", len, first, P, j);
    CHECK(p.stage_lo >= 0 && p.stage_hi <= n && p.stage_lo <= p.own_lo, "len %u P %d part %d", len, P, j);
    CHECK(p.stage_hi >= (p.own_hi + 16 < n ? p.own_hi + 16 : n), "len %u P %d part %d", len, P, j);
    for (int t = j * nl; t < (j + 1) * nl; ++t) {  // the lanes this part runs
      const int32_t start = n - (int32_t(tk::kSpanLanes) - t) * L;
      const int32_t b0 = start > c0 ? start : c0, b1 = start + L;  // bytes the lane folds
      if (b1 <= b0) continue;                                       // wholly before the CRC range
      CHECK(b0 >= p.own_lo && b1 <= p.own_hi, "lane %d [%d,%d) own [%d,%d) len %u P %d", t, b0, b1,
            p.own_lo, p.own_hi, len, P);
      CHECK(b0 >= p.stage_lo && b1 <= p.stage_hi, "lane %d not staged, len %u P %d", t, len, P);
    }
    prev = p.own_hi;
  }
  CHECK(prev == n, "len %u P %d: parts end at %d", len, P, prev);
  const tk::SpanPart one = tk::span_part(len, first, 1, 0);
  CHECK(one.own_lo == 0 && one.own_hi == n && one.stage_lo == 0 && one.stage_hi == n, "P 1 len %u", len);
}

int main() {
  uint64_t cases = 0;
  for (uint32_t len = 22; len <= tk::kSpanSegMax; len += len < 4096 ? 1 : 61) {
    for (int first = 0; first < 2; ++first)
      for (int P = 2; P <= 4; P += 2) {
        check(len, first != 0, P);
        ++cases;
      }
  }
  for (int first = 0; first < 2; ++first) {  // the lane-size boundary and the largest segment
    for (uint32_t len : {tk::kSpanLaneSmall * tk::kSpanLanes + 20u, tk::kSpanLaneSmall * tk::kSpanLanes + 21u,
                         tk::kSpanLaneSmall * tk::kSpanLanes + 22u, tk::kSpanSegMax})
      for (int P = 2; P <= 4; P += 2) check(len, first != 0, P);
  }
  std::printf("span_split_test: ok (%llu segment shapes)\n", static_cast<unsigned long long>(cases));
  return 0;
}
