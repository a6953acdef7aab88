// CRC32C (Castagnoli, reflected polynomial 0x82F63B78).
//
// Kafka's RecordBatch v2 protects attributes..end with CRC32C; kafka-python
// verifies it on every fetched batch when `check_crcs=True` (its default), so
// our consumer does the same.  On x86 the SSE4.2 `crc32` instruction has a
// 3-cycle latency and 1/cycle throughput: a single dependency chain reaches
// ~1/3 of the unit's rate, so long buffers are split into three independent
// streams whose raw states are merged with a GF(2) "shift by L zero bytes".
#include "crc32c.h"

#include "span.h"

#include <cstdlib>
#include <cstring>
#include <stdexcept>

#if defined(__x86_64__)
#include <immintrin.h>
#include <nmmintrin.h>
#include <xmmintrin.h>
#endif

namespace tk {
namespace {

constexpr uint32_t kPoly = 0x82F63B78u;

// ---- table (slicing-by-8) fallback -------------------------------------
struct Tables {
  uint32_t t[8][256];
  // x^(2^k) mod P in zlib's reflected representation (x^0 == 1<<31).
  uint32_t x2n[32];
  Tables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = t[0][i];
      for (int s = 1; s < 8; ++s) {
        c = t[0][c & 0xFF] ^ (c >> 8);
        t[s][i] = c;
      }
    }
    uint32_t p = 1u << 30;  // x^1
    x2n[0] = p;
    for (int n = 1; n < 32; ++n) x2n[n] = p = multmodp(p, p);
  }
  static uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
      if (a & m) {
        p ^= b;
        if ((a & (m - 1)) == 0) break;
      }
      m >>= 1;
      b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
  }
  // x^(n * 2^k) mod P
  uint32_t x2nmodp(uint64_t n, unsigned k) const {
    uint32_t p = 1u << 31;
    while (n) {
      if (n & 1) p = multmodp(x2n[k & 31], p);
      n >>= 1;
      ++k;
    }
    return p;
  }
};

const Tables& tables() {
  static const Tables t;
  return t;
}

uint32_t raw_sw(uint32_t s, const uint8_t* p, size_t n) {
  const auto& T = tables().t;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    s = T[0][(s ^ *p++) & 0xFF] ^ (s >> 8);
    --n;
  }
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    w ^= s;
    s = T[7][w & 0xFF] ^ T[6][(w >> 8) & 0xFF] ^ T[5][(w >> 16) & 0xFF] ^ T[4][(w >> 24) & 0xFF] ^
        T[3][(w >> 32) & 0xFF] ^ T[2][(w >> 40) & 0xFF] ^ T[1][(w >> 48) & 0xFF] ^ T[0][w >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) s = T[0][(s ^ *p++) & 0xFF] ^ (s >> 8);
  return s;
}

#if defined(__x86_64__)
// Block lengths for the 3-stream interleave and their shift constants.
constexpr size_t kBlocks[] = {8192, 1024, 128};
// Software prefetch distance (bytes) inside each stream (0 disables; TORCHKAFKA_CRC_PREFETCH).
const size_t kPrefetch = [] {
  const char* e = std::getenv("TORCHKAFKA_CRC_PREFETCH");
  return e ? size_t(std::strtoul(e, nullptr, 10)) : size_t(1024);
}();

struct ShiftConsts {
  uint32_t k[3];
  ShiftConsts() {
    for (int i = 0; i < 3; ++i) k[i] = tables().x2nmodp(kBlocks[i], 3);
  }
};
const ShiftConsts& shift_consts() {
  static const ShiftConsts c;
  return c;
}

__attribute__((target("sse4.2"))) inline uint32_t stream_hw(uint32_t s, const uint8_t* p, size_t n) {
  uint64_t c = s;
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    c = _mm_crc32_u64(c, w);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = uint32_t(c);
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}

__attribute__((target("sse4.2"))) uint32_t raw_hw(uint32_t s, const uint8_t* p, size_t n) {
  const auto& K = shift_consts();
  for (int bi = 0; bi < 3; ++bi) {
    const size_t L = kBlocks[bi];
    while (n >= 3 * L) {
      uint64_t a = s, b = 0, c = 0;
      const uint8_t* pa = p;
      const uint8_t* pb = p + L;
      const uint8_t* pc = p + 2 * L;
      for (size_t i = 0; i < L; i += 8) {
        if ((i & 63) == 0 && kPrefetch) {
          // the log is read cold from DRAM; the L2 streamer stops at 4 KiB page boundaries, so
          // keep each of the three streams' next lines requested ahead explicitly
          _mm_prefetch(reinterpret_cast<const char*>(pa + i + kPrefetch), _MM_HINT_T0);
          _mm_prefetch(reinterpret_cast<const char*>(pb + i + kPrefetch), _MM_HINT_T0);
          _mm_prefetch(reinterpret_cast<const char*>(pc + i + kPrefetch), _MM_HINT_T0);
        }
        uint64_t wa, wb, wc;
        std::memcpy(&wa, pa + i, 8);
        std::memcpy(&wb, pb + i, 8);
        std::memcpy(&wc, pc + i, 8);
        a = _mm_crc32_u64(a, wa);
        b = _mm_crc32_u64(b, wb);
        c = _mm_crc32_u64(c, wc);
      }
      // state(A||B||C) = shift(shift(a, L) ^ b, L) ^ c
      uint32_t ab = Tables::multmodp(K.k[bi], uint32_t(a)) ^ uint32_t(b);
      s = Tables::multmodp(K.k[bi], ab) ^ uint32_t(c);
      p += 3 * L;
      n -= 3 * L;
    }
  }
  return stream_hw(s, p, n);
}

bool detect_hw() { return __builtin_cpu_supports("sse4.2"); }

// ---- carry-less-multiply folding (AVX-512 VPCLMULQDQ) -------------------
// The crc32 instruction tops out at 8 bytes/cycle even with three streams (~27 GB/s on the
// MI355X host: a third of a worker's per-batch time in BASELINE config 2).  Folding instead
// keeps four 512-bit accumulators (16 independent 128-bit lanes) and advances each by 2048
// bits per step with two VPCLMULQDQ and one 3-way XOR: A' = lo(A) * k_lo ^ hi(A) * k_hi ^ next,
// where for a fold distance of D bits k_lo = (x^(D+32) mod P) << 1 and k_hi = (x^(D-32) mod P)
// << 1 in the reflected representation (derived and checked against the bitwise CRC; tests).
// The lanes are then folded into one 128-bit remainder whose raw CRC (two crc32 instructions
// from state 0) is the CRC of everything folded.
const size_t kFoldPrefetch = [] {
  const char* e = std::getenv("TORCHKAFKA_CRC_FOLD_PREFETCH");  // 512/1K/2K/4K: 45.3/45.3/45.4/45.9 M rec/s
  return e ? size_t(std::strtoul(e, nullptr, 10)) : size_t(4096);
}();

struct FoldConsts {
  __m128i k2048, k512, k384, k256, k128;
  FoldConsts() {
    auto k = [](unsigned D) {
      const uint64_t lo = uint64_t(tables().x2nmodp(D + 32, 0)) << 1;
      const uint64_t hi = uint64_t(tables().x2nmodp(D - 32, 0)) << 1;
      return _mm_set_epi64x(int64_t(hi), int64_t(lo));
    };
    k2048 = k(2048);
    k512 = k(512);
    k384 = k(384);
    k256 = k(256);
    k128 = k(128);
  }
};
const FoldConsts& fold_consts() {
  static const FoldConsts c;
  return c;
}

__attribute__((target("avx512f,vpclmulqdq"), always_inline)) inline __m512i fold512(__m512i a, __m512i k, __m512i b) {
  return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(a, k, 0x00), _mm512_clmulepi64_epi128(a, k, 0x11), b,
                                   0x96);
}
__attribute__((target("pclmul,sse4.1"), always_inline)) inline __m128i fold128(__m128i a, __m128i k) {
  return _mm_xor_si128(_mm_clmulepi64_si128(a, k, 0x00), _mm_clmulepi64_si128(a, k, 0x11));
}

// Needs n >= 256.
__attribute__((target("avx512f,avx512dq,vpclmulqdq,pclmul,sse4.2"))) uint32_t raw_fold(uint32_t s, const uint8_t* p,
                                                                                       size_t n) {
  const FoldConsts& C = fold_consts();
  __m512i a0 = _mm512_loadu_si512(p), a1 = _mm512_loadu_si512(p + 64), a2 = _mm512_loadu_si512(p + 128),
          a3 = _mm512_loadu_si512(p + 192);
  a0 = _mm512_xor_si512(a0, _mm512_castsi128_si512(_mm_cvtsi32_si128(int(s))));  // the running state
  p += 256;
  n -= 256;
  const __m512i k = _mm512_broadcast_i32x4(C.k2048);
  while (n >= 256) {
    // the log is usually read cold from DRAM: keep kFoldPrefetch bytes requested ahead
    _mm_prefetch(reinterpret_cast<const char*>(p + kFoldPrefetch), _MM_HINT_T0);
    _mm_prefetch(reinterpret_cast<const char*>(p + kFoldPrefetch + 64), _MM_HINT_T0);
    _mm_prefetch(reinterpret_cast<const char*>(p + kFoldPrefetch + 128), _MM_HINT_T0);
    _mm_prefetch(reinterpret_cast<const char*>(p + kFoldPrefetch + 192), _MM_HINT_T0);
    a0 = fold512(a0, k, _mm512_loadu_si512(p));
    a1 = fold512(a1, k, _mm512_loadu_si512(p + 64));
    a2 = fold512(a2, k, _mm512_loadu_si512(p + 128));
    a3 = fold512(a3, k, _mm512_loadu_si512(p + 192));
    p += 256;
    n -= 256;
  }
  const __m512i k5 = _mm512_broadcast_i32x4(C.k512);
  a1 = fold512(a0, k5, a1);
  a2 = fold512(a1, k5, a2);
  a3 = fold512(a2, k5, a3);
  __m128i x = _mm512_extracti64x2_epi64(a3, 3);
  x = _mm_xor_si128(x, fold128(_mm512_extracti64x2_epi64(a3, 0), C.k384));
  x = _mm_xor_si128(x, fold128(_mm512_extracti64x2_epi64(a3, 1), C.k256));
  x = _mm_xor_si128(x, fold128(_mm512_extracti64x2_epi64(a3, 2), C.k128));
  uint64_t r = _mm_crc32_u64(0, uint64_t(_mm_cvtsi128_si64(x)));
  r = _mm_crc32_u64(r, uint64_t(_mm_extract_epi64(x, 1)));
  return n ? raw_hw(uint32_t(r), p, n) : uint32_t(r);
}

bool detect_fold() {
  const char* e = std::getenv("TORCHKAFKA_CRC_FOLD");
  if (e && e[0] == '0') return false;
  return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
         __builtin_cpu_supports("vpclmulqdq") && __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.2");
}
#else
bool detect_hw() { return false; }
uint32_t raw_hw(uint32_t s, const uint8_t* p, size_t n) { return raw_sw(s, p, n); }
#endif

const bool g_hw = detect_hw();
#if defined(__x86_64__)
const bool g_fold = detect_fold();
constexpr size_t kFoldMin = 512;  // below this the 3-stream crc32 path is as fast
#endif

}  // namespace

bool crc32c_hw() { return g_hw; }
bool crc32c_fold() {
#if defined(__x86_64__)
  return g_fold;
#else
  return false;
#endif
}

uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  const auto* p = static_cast<const uint8_t*>(data);
  uint32_t s = ~crc;
#if defined(__x86_64__)
  if (g_fold && n >= kFoldMin) return ~raw_fold(s, p, n);
#endif
  s = g_hw ? raw_hw(s, p, n) : raw_sw(s, p, n);
  return ~s;
}

uint32_t crc32c_method(int method, const void* data, size_t n) {
  const auto* p = static_cast<const uint8_t*>(data);
  switch (method) {
    case 0: return ~raw_sw(~0u, p, n);
#if defined(__x86_64__)
    case 1: if (g_hw) return ~raw_hw(~0u, p, n); break;
    case 2: if (g_fold && n >= 256) return ~raw_fold(~0u, p, n); break;
#endif
    default: break;
  }
  throw std::invalid_argument("crc32c: method unavailable on this CPU / length");
}

uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }

// ---- device-decode support (span.h) --------------------------------------
uint32_t crc32c_shift_raw(uint32_t raw, uint64_t n_bytes) {
  const Tables& T = tables();
  return Tables::multmodp(T.x2nmodp(n_bytes, 3), raw);
}

void crc32c_span_tables(uint32_t* out) {
  const Tables& T = tables();
  for (int k = 0; k < 8; ++k)
    for (int b = 0; b < 256; ++b) out[kSpanTabSlice + k * 256 + b] = T.t[k][b];
  for (int k = 0; k < 8; ++k)
    for (int n = 0; n < 16; ++n) {
      out[kSpanTabNib + (2 * k) * 16 + n] = T.t[k][n];
      out[kSpanTabNib + (2 * k + 1) * 16 + n] = T.t[k][n << 4];
    }
  const uint32_t gap = T.x2nmodp(uint64_t(kSpanWin - kSpanPiece), 3);
  for (uint32_t i = 0; i < 8; ++i)
    for (uint32_t n = 0; n < 16; ++n) out[kSpanTabGap + i * 16 + n] = Tables::multmodp(gap, n << (4 * i));
  for (uint32_t m = 0; m < 32; ++m)
    for (uint32_t t = 0; t < kSpanLanes; ++t)
      out[kSpanTabLaneMul + m * kSpanLanes + t] =
          T.x2nmodp(uint64_t(kSpanPiece) * (kSpanLanes - 1 - t) + uint64_t(kSpanWin) * m, 3);
}

uint32_t crc32c_span_emulate(const uint8_t* buf, uint32_t c0, uint32_t c1, bool first, int parts) {
  // Host mirror of the device CRC stage (span_device.h), step for step: windows of kSpanWin bytes
  // ending at c1, lane t folding its kSpanPiece bytes of every window into a running state (the
  // window gap operator between windows), looked up in the same nibble rows; a slice-by-4 step for
  // a piece's first 4 bytes then slice-by-8 steps; bytes below c0 masked to zero (8-byte groups
  // wholly below c0 skipped); the first 4 CRC'd bytes of a RecordBatch xor 0xFF (the 0xFFFFFFFF
  // initial value); then every lane's state times its lane constant, xored.  The range is the
  // segment [0, c1) with c0 < 22.
  static uint32_t tab[kSpanTabWords];
  static const bool init = (crc32c_span_tables(tab), true);
  (void)init;
  auto byte_at = [&](int64_t ab) -> uint32_t {
    uint32_t b = ab >= int64_t(c0) ? buf[ab] : 0u;
    if (first && ab >= int64_t(c0) && ab < int64_t(c0) + 4) b ^= 0xFFu;
    return b;
  };
  auto word_at = [&](int64_t a) -> uint32_t {
    uint32_t w = 0;
    for (int k = 0; k < 4; ++k) w |= byte_at(a + k) << (8 * k);
    return w;
  };
  // byte table k through its two nibble rows, as the kernel looks it up (span_device.h nib_dword)
  const uint32_t* N = tab + kSpanTabNib;
  auto nib = [&](uint32_t w, int b) {
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
      const uint32_t v = (w >> (8 * i)) & 255u;
      r ^= N[(2 * (b - i)) * 16 + (v & 15u)] ^ N[(2 * (b - i) + 1) * 16 + (v >> 4)];
    }
    return r;
  };
  auto gap = [&](uint32_t c) {
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= tab[kSpanTabGap + i * 16 + ((c >> (4 * i)) & 15u)];
    return r;
  };
  const int64_t nw = int64_t(span_windows(c1));
  const int64_t w0 = int64_t(c1) - nw * int64_t(kSpanWin);
  // segment parts (span_device.h crc_finish): each part's windows from a zero state, each lane moved
  // to the segment's end (past the later lanes' pieces and the windows after the part's last), xored
  if (parts < 1) parts = 1;
  uint32_t total = 0;
  for (int q = 0; q < parts; ++q) {
  const int64_t k0 = span_part_k0(q, parts, int32_t(nw)), k1 = span_part_k0(q + 1, parts, int32_t(nw));
  uint32_t lane[kSpanLanes] = {};
  for (int64_t k = k0; k < k1; ++k) {
    for (uint32_t t = 0; t < kSpanLanes; ++t) {
      const int64_t start = w0 + k * int64_t(kSpanWin) + int64_t(t) * kSpanPiece;
      uint32_t crc = gap(lane[t]);
      if (start + 4 > int64_t(c0)) crc = nib(crc ^ word_at(start), 3);
      for (uint32_t j = 0; j < (kSpanPiece - 4) / 8; ++j) {
        const int64_t a = start + 4 + 8 * int64_t(j);
        if (a + 8 <= int64_t(c0)) continue;
        const uint32_t x = crc ^ word_at(a), y = word_at(a + 4);
        crc = nib(x, 7) ^ nib(y, 3);
      }
      lane[t] = crc;
    }
  }
  const uint32_t* K = tab + kSpanTabLaneMul + uint32_t(nw - k1) * kSpanLanes;
  for (uint32_t t = 0; t < kSpanLanes; ++t) total ^= Tables::multmodp(K[t], lane[t]);
  }
  return total;
}

}  // namespace tk
